// dgraph_amd — fp32 MFMA dual GEMM for the GraphSAGE combine at the reference's precision
// (gfx950, v_mfma_f32_16x16x4_f32: exact f32, a k-ordered fmaf chain per output).
//
//   out[o(i), :] = epi( A1[a(i), 0:K1] @ B1[K1, N] (+ A2[a(i), 0:K2] @ B2[K2, N]) )
//   epi(v) = relu?( gate?( rs[i] * v + bias[n] + beta * cin[o(i), n] ) )   (rs nullable)
//   gate: v = gate[o(i), n] > 0 ? v : 0   (the ReLU derivative read from an activation)
//   a(i) = a_rows ? a_rows[i] : i (A1 only; A2 is read densely), o(i) = o_rows ? o_rows[i] : i
//
// The reference runs these combines as two torch.mm calls plus adds (fp32 only,
// DGraph/distributed/csrc/torch_local_kernels.cu:43-46 and the experiments' nn.Linear
// layers). fp32 MFMA runs at the f32 vector rate (64 FLOP/clk/SIMD, 157 TF/s), so at
// K=256..512 the combine is COMPUTE bound (~64 FLOP per byte moved): the design goal is
// keeping the matrix pipe busy, and fusing the second GEMM, bias, ReLU and the gradient
// gate so no extra pass over an [M, N] fp32 tensor is spent.
//
// Tiling: 512 threads (8 waves, 2 per SIMD); a block owns BM = 256 rows x all N columns
// (A is read from HBM once); waves form a WM x WN grid, each with TM x TN 16x16 tiles
// (TM*TN*4 accumulator registers). K runs in 32-deep stages through two LDS buffers:
//   * A stage [256][32] fp32 (32 KB), B stage [32][N+4] fp32 (row pad: the 8-apart k rows
//     one b32 fragment read touches fall in different banks);
//   * stage s+1 is staged global -> LDS by LDS-DMA (global_load_lds_dwordx4: no staging
//     registers; 212-218 VGPRs instead of 240) into the other buffer while stage s's MFMAs
//     run, retired by vmcnt(0) + one barrier per stage. Measured against register staging,
//     against B-fragment reads pinned a whole MFMA step ahead, and against the next stage's
//     fragments prefetched behind the last MFMA step: all within +-0.3 % on the papers100M
//     step (profiles/r04/gemm_f32_staging_ab.log), so the simplest form is kept;
//   * k order inside a stage: lane group h = lane>>4 takes k = 8h + j in MFMA step j, so a
//     lane's A fragments of the stage are two 16-B pieces (2 x ds_read_b128) and its B
//     fragment of step j is row 8h + j (the permutation is applied to A and B alike; the
//     summation order stays fixed, so results are run-to-run identical);
//   * LDS bank conflicts removed: the A stage's 16-B chunks are XOR-swizzled per row pair
//     (a_chunk: every ds_read_b128 lane group touches 16 distinct 4-bank slots; the naive
//     layout was 4-way conflicted), B rows 8..15 and 24..31 of a stage sit 16 floats further
//     inside an (N+16)-float pitch
//     (the two 16-lane halves of a ds_read_b32 fall in opposite bank halves: was 2-way);
//   * persistent grid (one 512-thread block per CU) pulling 256-row tiles from a work
//     counter (dynamic: a block whose CU is held by another kernel, e.g. RCCL's during a
//     halo exchange, starts late and finds the tiles taken, instead of running its static
//     share after everyone else); tile indices are fetched a tile ahead, and the next
//     tile's first stage is loaded during the current tile's last stage, so the prologue's
//     global latency and the epilogue's stores overlap MFMAs.
#include "../common.h"
#include "kernels.h"
#include "lds_dma.h"

#include <mutex>
#include <unordered_map>

namespace dgraph {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBK = 32;


// Block shape: BM = 256 rows, 512 threads (8 waves, 2 per SIMD at ~240 VGPRs): the GEMM owns
// the whole register file of the CU (a 128-row one-wave-per-SIMD variant meant to co-reside
// with the aggregation measured slower and was removed, PERFORMANCE.md).
template <int BM, int N>
struct GCfg;
// (BM, N): (TM, TN, WM, WN) with 16*TM*WM = BM and 16*TN*WN = N; threads = 64*WM*WN
// (a 4-wave block with a 128 x 128 tile per wave — 256 accumulators, one wave per SIMD —
// compiles to 256 VGPRs + 256 AGPRs with scratch spills on gfx950/hipcc 7.2: not used)
template <> struct GCfg<256, 256> { static constexpr int TM = 4, TN = 8, WM = 4, WN = 2; };
template <> struct GCfg<256, 192> { static constexpr int TM = 4, TN = 6, WM = 4, WN = 2; };
template <> struct GCfg<256, 176> { static constexpr int TM = 2, TN = 11, WM = 8, WN = 1; };
template <> struct GCfg<256, 128> { static constexpr int TM = 2, TN = 8, WM = 8, WN = 1; };
template <> struct GCfg<256, 64> { static constexpr int TM = 2, TN = 4, WM = 8, WN = 1; };
template <int BM, int N>
constexpr int threads_of() { return 64 * GCfg<BM, N>::WM * GCfg<BM, N>::WN; }

// A stage: 16-B chunk c of row r lives at chunk a_chunk(r, c) of the row (XOR swizzle by
// row pair; table found by exhaustive search over the ds_read_b128 lane groups)
constexpr uint32_t kASwz = 0x32765410u;
__device__ __forceinline__ int a_chunk(int r, int c) {
  return c ^ static_cast<int>((kASwz >> (4 * ((r >> 1) & 7))) & 7u);
}

template <int BM, int N>
struct GLds {
  static constexpr int kThreads = threads_of<BM, N>();
  static constexpr int BP = N + 16;  // B stage row pitch (floats): room for b_row's shift
  static constexpr int A_FL = BM * kBK;                 // A stage floats
  static constexpr int B_FL = kBK * BP;                 // B stage floats
  static constexpr int STAGE = A_FL + B_FL;
  static constexpr size_t BYTES = 2 * STAGE * sizeof(float);
};

// B stage row k starts at b_row(k): rows with bit 3 set are shifted by 16 floats
template <int BP>
__device__ __forceinline__ int b_row(int k) { return k * BP + ((k >> 3) & 1) * 16; }

template <int BM, int N, bool HAS_A2, bool RELU, bool HAS_BIAS, bool HAS_CIN, bool HAS_GATE>
__device__ __forceinline__ void gemm_f32_body(
    const float* __restrict__ A1, int64_t lda1, int K1, const float* __restrict__ B1,
    int64_t ldb1, const float* __restrict__ A2, int64_t lda2, int K2,
    const float* __restrict__ B2, int64_t ldb2, const int64_t* __restrict__ a_rows,
    const float* __restrict__ bias, const float* cin, int64_t ldc, float beta,
    const float* __restrict__ gate, int64_t ldg, const int64_t* __restrict__ o_rows,
    const float* __restrict__ row_scale, float* out, int64_t ldo, int64_t M,
    int* __restrict__ tile_ctr, float* __restrict__ send_out, int64_t lds_send,
    const int64_t* __restrict__ send_ptr, const int32_t* __restrict__ send_pos) {
  constexpr int kBM = BM;
  using C = GCfg<BM, N>;
  using L = GLds<BM, N>;
  constexpr int kThreads = L::kThreads;
  static_assert(64 * C::WM * C::WN == kThreads, "waves x 64 == threads");
  constexpr int TM = C::TM, TN = C::TN, WN = C::WN;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 15;  // fragment row (A) / column (B, C)
  const int lh = lane >> 4;  // k slot group
  const int K = K1 + K2;
  const int nst = K / kBK;
  const int64_t ntiles = (M + kBM - 1) / kBM;
  __shared__ int s_tile;
  // tile_ctr == nullptr: static schedule (block b walks tiles b, b + grid, ...). Dynamic:
  // thread 0 keeps ONE counter fetch in flight a whole tile ahead (``pending``) and
  // publishes it through LDS at the top of the next tile, so the atomic's latency is never
  // waited for; readfirstlane keeps the block-uniform indices in scalar registers
  const bool dyn = tile_ctr != nullptr;
  int pending = 0;
  if (dyn) {
    if (tid == 0) {
      s_tile = atomicAdd(tile_ctr, 1);
      pending = atomicAdd(tile_ctr, 1);
    }
    __syncthreads();
  }
  int64_t tile = dyn ? __builtin_amdgcn_readfirstlane(s_tile) : blockIdx.x;
  if (tile >= ntiles) return;  // block-uniform

  // ---- LDS-DMA staging of a stage (no staging registers): wave w issues 4 A pieces
  // (piece P = 4w + u = rows 8P..8P+7 of the tile, 1 KB, lane l -> row 8P + l/8, LDS slot
  // l%8 of the row, which holds global chunk (l%8) ^ swz(row): the A swizzle moved to the
  // per-lane SOURCE address) and 4 B rows (row kr = 4w + u, lane l < N/4 -> columns
  // 4l..4l+3). Row indices are 32-bit (the launcher checks every operand has < 2^31 rows).
  constexpr int NW = kThreads / 64;  // waves
  constexpr int PW = 32 / NW;         // A pieces and B rows per wave per stage
  static_assert(32 % NW == 0 && kBM == 256 && kBK == 32, "staging map");
  int32_t a_src_row[PW];   // A1 rows of the tile being loaded (through a_rows)
  int32_t nx_src_row[PW];  // the next tile's A1 rows (index loads issued early)
  int64_t ld_tile = tile; // the tile whose stages issue_stage reads (A2 rows dense)
  const int a_slot = lane & 7;
  auto rows_of = [&](int64_t t, int32_t* a1) {
#pragma unroll
    for (int u = 0; u < PW; ++u) {
      int64_t r = t * kBM + (PW * wave + u) * 8 + (lane >> 3);
      r = r < M ? r : M - 1;  // rows past M read a valid row (never stored)
      a1[u] = static_cast<int32_t>(a_rows ? a_rows[r] : r);
    }
  };
  rows_of(tile, a_src_row);
  auto issue_stage = [&](int s, int buf) {
    const int k0 = s * kBK;
    const bool first = !HAS_A2 || k0 < K1;
    const float* Ab = first ? A1 : A2;
    const int64_t lda = first ? lda1 : lda2;
    const int ka = first ? k0 : k0 - K1;
    float* sa = lds + buf * L::STAGE;
    float* sb = sa + L::A_FL;
#pragma unroll
    for (int u = 0; u < PW; ++u) {
      const int r = (PW * wave + u) * 8 + (lane >> 3);  // row within the tile
      int64_t r2 = ld_tile * kBM + r;
      r2 = r2 < M ? r2 : M - 1;
      const int64_t ar = first ? static_cast<int64_t>(a_src_row[u]) : r2;
      const int c = a_chunk(r, a_slot);  // XOR swizzle: its own inverse
      glds16(Ab + ar * lda + ka + c * 4, sa + (PW * wave + u) * 8 * kBK);
    }
    const float* Bb = first ? B1 : B2;
    const int64_t ldb = first ? ldb1 : ldb2;
#pragma unroll
    for (int u = 0; u < PW; ++u) {
      const int kr = PW * wave + u;
      if (lane < N / 4)
        glds16(Bb + static_cast<int64_t>(ka + kr) * ldb + lane * 4, sb + b_row<L::BP>(kr));
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_stage(0, 0);
  wait_vmcnt<0>();
  __syncthreads();
  const int arow_w = wm * TM * 16;  // this wave's first row within the block tile
  const int bcol_w = wn * TN * 16;  // this wave's first column
  int g = 0;                        // stages run by this block (LDS buffer parity)
  while (true) {
    int64_t next = tile + gridDim.x;
    if (dyn) {
      if (tid == 0) {
        s_tile = pending;  // fetched a tile ago
        pending = atomicAdd(tile_ctr, 1);
      }
      __syncthreads();
      next = __builtin_amdgcn_readfirstlane(s_tile);
    }
    const bool has_next = next < ntiles;  // block-uniform
    rows_of(has_next ? next : tile, nx_src_row);  // consumed at the tile's last stage
    for (int s = 0; s < nst; ++s, ++g) {
      const int buf = g & 1;
      // the next stage, in flight during this stage's MFMAs; at the tile's last stage the
      // next tile's first stage (or, for the block's last tile, a harmless re-read of this
      // tile's first stage). Branch-free: every path issues the same loads into the same
      // registers, so no wait is forced before the MFMAs below.
      const bool last = s + 1 == nst;
      const bool switch_tile = last && has_next;
#pragma unroll
      for (int u = 0; u < PW; ++u) a_src_row[u] = switch_tile ? nx_src_row[u] : a_src_row[u];
      ld_tile = switch_tile ? next : ld_tile;
      // the other buffer was last read in the previous stage (before its barrier)
      issue_stage(last ? 0 : s + 1, buf ^ 1);
      __builtin_amdgcn_sched_barrier(0);
      const float* sa = lds + buf * L::STAGE;
      const float* sb = sa + L::A_FL;
      // A fragments of the whole stage: k = 8 lh .. 8 lh + 7 of row (tile a, li)
      f32x4 af[TM][2];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int r = arow_w + a * 16 + li;
        const float* p = sa + r * kBK;
        af[a][0] = *reinterpret_cast<const f32x4*>(p + a_chunk(r, 2 * lh) * 4);
        af[a][1] = *reinterpret_cast<const f32x4*>(p + a_chunk(r, 2 * lh + 1) * 4);
      }
      const float* sbw = sb + b_row<L::BP>(8 * lh) + bcol_w + li;
      {
        // B fragments double-buffered across MFMA steps: step j+1's LDS reads are issued
        // before step j's TM*TN MFMAs
        float bf[2][TN];
#pragma unroll
        for (int b = 0; b < TN; ++b) bf[0][b] = sbw[b * 16];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (j + 1 < 8) {
#pragma unroll
            for (int b = 0; b < TN; ++b) bf[(j + 1) & 1][b] = sbw[(j + 1) * L::BP + b * 16];
          }
#pragma unroll
          for (int a = 0; a < TM; ++a) {
            const float av = af[a][j >> 2][j & 3];
#pragma unroll
            for (int b = 0; b < TN; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bf[j & 1][b], acc[a][b], 0, 0, 0);
          }
        }
      }
      // this stage's DMAs landed (the block's very last ones fill a buffer never read)
      wait_vmcnt<0>();
      __syncthreads();
    }

    // ---- epilogue: tile (a, b) register r of lane l is element
    //      (row 4 (l >> 4) + r, column l & 15) of the 16x16 block
    const int64_t row0 = tile * kBM;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t i = row0 + arow_w + a * 16 + 4 * lh + r;
        if (i < M) {
          const int64_t orow = o_rows ? o_rows[i] : i;
          const float rsc = row_scale ? row_scale[i] : 1.f;
          // the row's cin / gate operands loaded together before any store: cin may alias
          // out (in place), so the compiler cannot move a later load above an earlier store
          // and each load would wait out its own latency. Safe in place: this thread reads
          // exactly the elements it writes, and no other thread touches them
          float cv[TN], gv[TN];
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            const int n = bcol_w + b * 16 + li;
            if constexpr (HAS_CIN) cv[b] = cin[orow * ldc + n];
            if constexpr (HAS_GATE) gv[b] = gate[orow * ldg + n];
          }
          float vals[TN];
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            const int n = bcol_w + b * 16 + li;
            float v = acc[a][b][r] * rsc;
            if constexpr (HAS_BIAS) v += bias[n];
            if constexpr (HAS_CIN) v = fmaf(beta, cv[b], v);
            if constexpr (HAS_GATE) v = gv[b] > 0.f ? v : 0.f;
            if constexpr (RELU) v = v > 0.f ? v : 0.f;
            out[orow * ldo + n] = v;
            vals[b] = v;
          }
          if (send_out != nullptr) {
            // the halo pack fused into the producer: the row also goes to each of its
            // positions in the exchange's send buffer (one per peer that needs it)
            const int64_t p1 = send_ptr[i + 1];
            for (int64_t q = send_ptr[i]; q < p1; ++q) {
              float* so = send_out + static_cast<int64_t>(send_pos[q]) * lds_send;
#pragma unroll
              for (int b = 0; b < TN; ++b) so[bcol_w + b * 16 + li] = vals[b];
            }
          }
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b][r] = 0.f;
      }
    }
    if (!has_next) break;
    tile = next;
  }
}

#define DG_GEMM_F32_ARGS                                                                        \
  const float *__restrict__ A1, int64_t lda1, int K1, const float *__restrict__ B1,          \
      int64_t ldb1, const float *__restrict__ A2, int64_t lda2, int K2,                       \
      const float *__restrict__ B2, int64_t ldb2, const int64_t *__restrict__ a_rows,         \
      const float *__restrict__ bias, const float *cin, int64_t ldc, float beta,              \
      const float *__restrict__ gate, int64_t ldg, const int64_t *__restrict__ o_rows,        \
      const float *__restrict__ row_scale, float *out, int64_t ldo, int64_t M, int *tile_ctr, \
      float *send_out, int64_t lds_send, const int64_t *send_ptr, const int32_t *send_pos
#define DG_GEMM_F32_PASS                                                                       \
  A1, lda1, K1, B1, ldb1, A2, lda2, K2, B2, ldb2, a_rows, bias, cin, ldc, beta, gate, ldg,     \
      o_rows, row_scale, out, ldo, M, tile_ctr, send_out, lds_send, send_ptr, send_pos

template <int N, bool HAS_A2, bool RELU, bool HAS_BIAS, bool HAS_CIN, bool HAS_GATE>
__global__ __launch_bounds__((threads_of<256, N>()), 1) void gemm_f32_kernel(DG_GEMM_F32_ARGS) {
  gemm_f32_body<256, N, HAS_A2, RELU, HAS_BIAS, HAS_CIN, HAS_GATE>(DG_GEMM_F32_PASS);
  work_counter_release(tile_ctr);
}

// the fused halo pack of the next gemm_f32 call (set_gemm_f32_send; host-side, one call)
GemmSend g_gemm_send;

template <int N, bool HAS_A2, bool RELU, bool HAS_BIAS, bool HAS_CIN, bool HAS_GATE>
hipError_t launch_gemm_f32(const float* A1, int64_t lda1, int K1, const float* B1, int64_t ldb1,
                           const float* A2, int64_t lda2, int K2, const float* B2,
                           int64_t ldb2, const int64_t* a_rows, const float* bias,
                           const float* cin, int64_t ldc, float beta, const float* gate,
                           int64_t ldg, const int64_t* o_rows, const float* rsc, float* out,
                           int64_t ldo, int64_t M, hipStream_t st) {
  auto kern = &gemm_f32_kernel<N, HAS_A2, RELU, HAS_BIAS, HAS_CIN, HAS_GATE>;
  constexpr int kBM = 256;
  constexpr size_t lds = GLds<256, N>::BYTES;
  static_assert(lds <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    attr = true;
  }
  static int num_cus = 0;
  if (num_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&num_cus, hipDeviceAttributeMultiprocessorCount, dev) !=
            hipSuccess || num_cus <= 0)
      num_cus = 256;
  }
  // persistent: one block per CU (LDS-limited), each pulling tiles from the work counter
  const int64_t ntiles = (M + kBM - 1) / kBM;
  const int64_t blocks = ntiles < num_cus ? ntiles : num_cus;
  int* ctr = nullptr;
  if (g_f32_dynamic) {
    // no free slot (more than the captured-launch budget recorded into graphs, or more
    // streams than slots): the static tile schedule of the same kernel (ctr == nullptr),
    // identical results, instead of failing the launch
    ctr = work_counter(st);
  }
  const GemmSend& sd = g_gemm_send;
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(blocks)), dim3((threads_of<256, N>())), lds, st, A1,
                     lda1, K1, B1, ldb1, A2, lda2, K2, B2, ldb2, a_rows, bias, cin, ldc, beta,
                     gate, ldg, o_rows, rsc, out, ldo, M, ctr, sd.out, sd.ld, sd.ptr, sd.pos);
  return hipGetLastError();
}

template <int N, bool HAS_A2, bool RELU>
hipError_t gemm_f32_flags(const float* A1, int64_t lda1, int K1, const float* B1, int64_t ldb1,
                          const float* A2, int64_t lda2, int K2, const float* B2, int64_t ldb2,
                          const int64_t* a_rows, const float* bias, const float* cin,
                          int64_t ldc, float beta, const float* gate, int64_t ldg,
                          const int64_t* o_rows, const float* rsc, float* out, int64_t ldo,
                          int64_t M, hipStream_t st) {
#define DG_GF(HB_, HC_, HG_)                                                                  \
  return launch_gemm_f32<N, HAS_A2, RELU, HB_, HC_, HG_>(A1, lda1, K1, B1, ldb1, A2, lda2, K2, \
                                                         B2, ldb2, a_rows, bias, cin, ldc,   \
                                                         beta, gate, ldg, o_rows, rsc, out,  \
                                                         ldo, M, st);
  const bool hb = bias != nullptr, hc = cin != nullptr, hg = gate != nullptr;
  if (hb && !hc && !hg) { DG_GF(true, false, false) }
  if (!hb && !hc && !hg) { DG_GF(false, false, false) }
  if (!hb && hc && !hg) { DG_GF(false, true, false) }
  if (!hb && hc && hg) { DG_GF(false, true, true) }
  if (!hb && !hc && hg) { DG_GF(false, false, true) }
  if (hb && hc && !hg) { DG_GF(true, true, false) }
  if (hb && !hc && hg) { DG_GF(true, false, true) }
  DG_GF(true, true, true)
#undef DG_GF
}

template <int N>
hipError_t gemm_f32_n(const float* A1, int64_t lda1, int K1, const float* B1, int64_t ldb1,
                      const float* A2, int64_t lda2, int K2, const float* B2, int64_t ldb2,
                      const int64_t* a_rows, const float* bias, const float* cin, int64_t ldc,
                      float beta, const float* gate, int64_t ldg, const int64_t* o_rows,
                      const float* rsc, bool relu, float* out, int64_t ldo, int64_t M,
                      hipStream_t st) {
#define DG_GN(A2_, R_)                                                                     \
  return gemm_f32_flags<N, A2_, R_>(A1, lda1, K1, B1, ldb1, A2, lda2, K2, B2, ldb2, a_rows, \
                                    bias, cin, ldc, beta, gate, ldg, o_rows, rsc, out, ldo, M, st);
  const bool two = A2 != nullptr && K2 > 0;
  if (two) {
    if (relu) { DG_GN(true, true) }
    DG_GN(true, false)
  }
  if (relu) { DG_GN(false, true) }
  DG_GN(false, false)
#undef DG_GN
}

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

bool g_f32_dynamic = true;
void set_f32_dynamic(bool on) { g_f32_dynamic = on; }
void set_gemm_f32_send(const GemmSend& s) { g_gemm_send = s; }

namespace {
constexpr int kCtrStreams = 1024;    // eager slots: one per stream
constexpr int kCtrCaptured = 3072;   // one per launch recorded into a HIP graph
constexpr int kCtrSlots = kCtrStreams + kCtrCaptured;
constexpr int kCtrStride = 16;       // ints per slot (64 B: one slot per cache line)
int* g_ctr_ring[64] = {nullptr};
std::mutex g_ctr_mu;
std::unordered_map<hipStream_t, int> g_ctr_slot[64];
int g_ctr_captured[64] = {0};

hipError_t ctr_ring(int dev) {
  if (g_ctr_ring[dev] != nullptr) return hipSuccess;
  const size_t bytes = static_cast<size_t>(kCtrSlots) * kCtrStride * sizeof(int);
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&g_ctr_ring[dev]), bytes);
  if (e != hipSuccess) {
    g_ctr_ring[dev] = nullptr;
    return e;
  }
  return hipMemset(g_ctr_ring[dev], 0, bytes);  // synchronous: zero before any launch
}
}  // namespace

hipError_t work_counters_init() {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lk(g_ctr_mu);
  return ctr_ring(dev);
}

int* work_counter(hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cap) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_ctr_mu);
  if (ctr_ring(dev) != hipSuccess) return nullptr;
  int slot;
  if (cap == hipStreamCaptureStatusActive) {
    // a launch recorded into a graph gets a slot of its own, never shared with eager
    // launches: a replay may run on any stream, concurrently with eager kernels of the
    // capturing stream (the kernel's last block re-zeroes it for the next replay)
    if (g_ctr_captured[dev] >= kCtrCaptured) return nullptr;
    slot = kCtrStreams + g_ctr_captured[dev]++;
  } else {
    auto& m = g_ctr_slot[dev];
    auto it = m.find(st);
    if (it == m.end()) {
      if (static_cast<int>(m.size()) >= kCtrStreams) return nullptr;  // more streams than slots
      it = m.emplace(st, static_cast<int>(m.size())).first;
    }
    slot = it->second;
  }
  // zero at every launch boundary of the slot's stream / graph node: the previous kernel's
  // last block reset it
  return g_ctr_ring[dev] + static_cast<size_t>(slot) * kCtrStride;
}

bool gemm_f32_supported(int64_t N, int64_t K1, int64_t K2) {
  return (N == 64 || N == 128 || N == 176 || N == 192 || N == 256) && K1 > 0 &&
         K1 % kBK == 0 && K2 >= 0 && K2 % kBK == 0;
}

hipError_t gemm_f32(const float* A1, int64_t lda1, int64_t K1, const float* B1, int64_t ldb1,
                    const float* A2, int64_t lda2, int64_t K2, const float* B2, int64_t ldb2,
                    const int64_t* a_rows, const float* bias, const float* cin, int64_t ldc,
                    float beta, const float* gate, int64_t ldg, const int64_t* o_rows,
                    const float* row_scale, bool relu, float* out, int64_t ldo, int64_t M,
                    int64_t N, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (!gemm_f32_supported(N, K1, A2 ? K2 : 0)) return hipErrorInvalidValue;
  if (!al16(A1) || lda1 % 4 || !al16(B1) || ldb1 % 4) return hipErrorInvalidValue;
  if (A2 && K2 > 0 && (!al16(A2) || lda2 % 4 || !al16(B2) || ldb2 % 4))
    return hipErrorInvalidValue;
  const int k1 = static_cast<int>(K1), k2 = A2 ? static_cast<int>(K2) : 0;
  switch (N) {
    case 256: return gemm_f32_n<256>(A1, lda1, k1, B1, ldb1, A2, lda2, k2, B2, ldb2, a_rows, bias, cin, ldc, beta, gate, ldg, o_rows, row_scale, relu, out, ldo, M, st);
    case 192: return gemm_f32_n<192>(A1, lda1, k1, B1, ldb1, A2, lda2, k2, B2, ldb2, a_rows, bias, cin, ldc, beta, gate, ldg, o_rows, row_scale, relu, out, ldo, M, st);
    case 176: return gemm_f32_n<176>(A1, lda1, k1, B1, ldb1, A2, lda2, k2, B2, ldb2, a_rows, bias, cin, ldc, beta, gate, ldg, o_rows, row_scale, relu, out, ldo, M, st);
    case 128: return gemm_f32_n<128>(A1, lda1, k1, B1, ldb1, A2, lda2, k2, B2, ldb2, a_rows, bias, cin, ldc, beta, gate, ldg, o_rows, row_scale, relu, out, ldo, M, st);
    default: return gemm_f32_n<64>(A1, lda1, k1, B1, ldb1, A2, lda2, k2, B2, ldb2, a_rows, bias, cin, ldc, beta, gate, ldg, o_rows, row_scale, relu, out, ldo, M, st);
  }
}

}  // namespace dgraph
