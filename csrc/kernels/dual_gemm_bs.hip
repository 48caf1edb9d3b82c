// dgraph_amd — "B-stationary" MFMA dual GEMM for the GraphSAGE layer combine (gfx950).
//
//   out[M, N] = epi( A1[M, K1] @ B1[K1, N]  (+ A2[M, K2] @ B2[K2, N])  (+ bias) (+ Cin) )
//
// Same contract and "tile32" mask layout as dual_gemm.hip, different data flow. The
// column-half design there keeps half of B^T in LDS and lets TWO blocks read every A row
// (one per column half), counting on the second read hitting the XCD's L2; on the
// papers100M combine shapes it ran at ~3.3 TB/s of unique bytes (A read + out write).
//
// Here every A row is read from HBM exactly once:
//   * a block has NT = N/32 waves; wave t keeps B[:, 32t .. 32t+31] in VGPRs for the whole
//     run (K/4 registers per lane: 128 at K=512) — the weights never touch LDS;
//   * the block streams 32-row A tiles (and, when present, the Cin tile and the input
//     keep-mask words) global -> LDS by LDS-DMA (global_load_lds_dwordx4, no staging
//     VGPRs) into NBUF rotating buffers, NBUF-1 tiles ahead of the MFMAs; completion is a
//     COUNTED s_waitcnt vmcnt (every wave issues the same number of DMAs per tile, so the
//     count is a compile-time constant) + a raw s_barrier, so the DMAs of later tiles
//     stay in flight across the barrier;
//   * LDS image of a tile: one 1024-B DMA "piece" per 1 KB of rows, pieces 16 B apart
//     (1040-B stride). K=512: a piece is one row. K<=256: a piece holds two 512-B row
//     slots and the odd row's 16-B chunks are XOR-swizzled by 8 (done on the per-lane
//     SOURCE address: the DMA writes lane-linear). Either way the 32 rows read by one
//     v_mfma_f32_32x32x16_bf16 A-fragment ds_read_b128 fall in distinct bank groups;
//   * each wave multiplies the shared A tile by its register-resident B columns (K/16
//     MFMAs into one 32x32 accumulator); epilogue (bias, Cin, input mask, ReLU + keep-mask
//     ballot) through a private LDS tile -> 16-B row-segment stores.
// Persistent grid (occupancy x CUs), tiles round-robin over blocks.
#include "../common.h"
#include "kernels.h"
#include "lds_dma.h"

namespace dgraph {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ bf16x8 as_bf16x8_bs(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

constexpr int kTR = 32;       // rows per tile (one MFMA row block)
constexpr int kEWs = 40;      // epilogue tile row (32 + 8 pad, elements)
constexpr int kPiece = 1040;  // LDS stride of one 1 KB DMA piece (+16 B: bank rotation)
constexpr int kLdsMax = 160 * 1024;

// wait until at most BASE + n * STEP vector-memory ops are outstanding, n = min(i, MAXN)
template <int BASE, int STEP, int MAXN>
__device__ __forceinline__ void wait_vmcnt_dyn(int64_t i) {
  if constexpr (MAXN == 0) {
    wait_vmcnt<BASE>();
  } else {
    if (i >= MAXN) wait_vmcnt<BASE + MAXN * STEP>();
    else wait_vmcnt_dyn<BASE, STEP, MAXN - 1>(i);
  }
}

template <int NT, int K, bool HC, bool HM>
struct BsCfg {
  static constexpr int KS = K / 16;
  static constexpr int RPI = K <= 256 ? 2 : 1;    // A rows per 1 KB piece
  static constexpr int INS_A = kTR / RPI;         // A pieces per tile
  static constexpr int JA = (INS_A + NT - 1) / NT;  // A DMAs per wave per tile
  static constexpr int A_BYTES = INS_A * kPiece;
  static constexpr int C_BYTES = HC ? 64 * 32 * NT : 0;  // Cin tile [32][N] bf16, linear
  static constexpr int M_BYTES = HM ? 128 * NT : 0;      // 16 mask words per wave
  static constexpr int BUF = (A_BYTES + C_BYTES + M_BYTES + 15) / 16 * 16;
  static constexpr int FIXED = NT * 32 * kEWs * 2 + 1024;  // epilogue tiles + DMA sink
  static constexpr int NBUF_FIT = (kLdsMax - FIXED) / BUF;
  // deep enough to cover HBM latency under load at one 8-wave block per CU (the LDS
  // budget allows one): 7 tiles ahead at K <= 256, 3 at K = 512
  static constexpr int NBUF = NBUF_FIT >= 8 ? 8 : NBUF_FIT;
  static constexpr int OPS = JA + (HC ? 2 : 0) + (HM ? 1 : 0);  // DMAs per wave per tile
  static constexpr int STORES_MIN = 2;  // out-row stores per wave per tile (lower bound)
  static constexpr size_t LDS = static_cast<size_t>(NBUF) * BUF + FIXED;
  static_assert(NBUF >= 2, "LDS budget");
  static_assert(K == 192 || K == 256 || K == 512, "row slot layout");
};

template <int NT, int K, bool HC, bool HM, bool RELU>
__global__ __launch_bounds__(NT * 64) void dual_gemm_bs_kernel(
    const uint16_t* __restrict__ A1, int64_t lda1, int K1, const uint16_t* __restrict__ B1t,
    const uint16_t* __restrict__ A2, int64_t lda2, const uint16_t* __restrict__ B2t,
    const float* __restrict__ bias, const uint16_t* __restrict__ cin, int64_t ldc,
    uint16_t* __restrict__ out, int64_t ldo, uint64_t* __restrict__ mask_out,
    const uint64_t* __restrict__ mask_in, int64_t M) {
  using C = BsCfg<NT, K, HC, HM>;
  constexpr int KS = C::KS, NBUF = C::NBUF;
  constexpr int N = NT * 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;  // = this wave's 32-column tile
  const int h = lane >> 5;
  const int col_l = lane & 31;
  uint16_t* const sE =
      reinterpret_cast<uint16_t*>(lds + NBUF * C::BUF) + wave * (32 * kEWs);
  unsigned char* const sink = lds + NBUF * C::BUF + NT * 32 * kEWs * 2;
  const int K2 = K - K1;

  // ---- stationary B columns of this wave: B[k][32 wave + col_l] for k = 16 s + 8 h + j
  bf16x8 bfr[KS];
  const int n = wave * 32 + col_l;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 16 * s + 8 * h;
    const uint16_t* src = k < K1 ? B1t + static_cast<int64_t>(n) * K1 + k
                                 : B2t + static_cast<int64_t>(n) * K2 + (k - K1);
    bfr[s] = as_bf16x8_bs(*reinterpret_cast<const uint4*>(src));
  }
  const float bv = bias ? bias[n] : 0.f;

  const int64_t ntiles = (M + kTR - 1) / kTR;
  const int64_t G = gridDim.x;
  const int64_t t0 = blockIdx.x;
  if (t0 >= ntiles) return;

  // ---- this lane's part of every A DMA: (row within the piece, logical 16-B chunk)
  // RPI == 1: the piece is one row, chunk = lane. RPI == 2: lanes 0-31 fill the even row's
  // 512-B slot, lanes 32-63 the odd row's, whose chunk q is stored at position q ^ 8.
  const int a_sub = C::RPI == 2 ? h : 0;
  const int a_q = C::RPI == 2 ? (col_l ^ (8 * h)) : lane;
  const bool a_on = a_q * 8 < K;  // K=192: chunks 24..31 of a 512-B slot stay empty
  const int a_k = a_q * 8;
  // per-lane DMA source bases (A1 or A2 by the lane's k) and byte strides, hoisted out of
  // the tile loop: a DMA's source is base + min(row, M-1) * stride
  const unsigned char* a_base = a_k < K1
      ? reinterpret_cast<const unsigned char*>(A1 + a_k)
      : reinterpret_cast<const unsigned char*>(A2 + (a_k - K1));
  const uint64_t a_ld = static_cast<uint64_t>(a_k < K1 ? lda1 : lda2) * 2;
  int a_row[C::JA];
  int a_dst[C::JA];  // byte offset of the piece in a buffer, or -1: the sink
#pragma unroll
  for (int j = 0; j < C::JA; ++j) {
    const int ii = wave + NT * j;
    const bool real = ii < C::INS_A;
    const int iv = real ? ii : C::INS_A - 1;
    a_row[j] = iv * C::RPI + a_sub;
    a_dst[j] = real ? iv * kPiece : -1;
  }
  const int64_t Mm1 = M - 1;
  // Cin pieces (HC): this lane's (row, column) inside the [32][N] tile image
  const int c_rr0 = ((2 * wave) * 1024 + 16 * lane) / (2 * N);
  const int c_cc0 = (((2 * wave) * 1024 + 16 * lane) % (2 * N)) / 2;
  const int c_rr1 = ((2 * wave + 1) * 1024 + 16 * lane) / (2 * N);
  const int c_cc1 = (((2 * wave + 1) * 1024 + 16 * lane) % (2 * N)) / 2;
  // DMAs of tile `tile` into buffer `b`; every wave issues exactly C::OPS (surplus A slots
  // re-load the last piece into the sink)
  auto issue_tile = [&](int64_t tile, int b) {
    unsigned char* base = lds + b * C::BUF;
    const int64_t r0 = tile * kTR;
#pragma unroll
    for (int j = 0; j < C::JA; ++j) {
      int64_t r = r0 + a_row[j];
      r = r < Mm1 ? r : Mm1;  // rows past M (and past the last tile) read a valid row
      unsigned char* dst = a_dst[j] >= 0 ? base + a_dst[j] : sink;
      if (a_on) glds16(a_base + static_cast<uint64_t>(r) * a_ld, dst);
    }
    if constexpr (HC) {
      int64_t r = r0 + c_rr0;
      r = r < Mm1 ? r : Mm1;
      glds16(cin + r * ldc + c_cc0, base + C::A_BYTES + (2 * wave) * 1024);
      r = r0 + c_rr1;
      r = r < Mm1 ? r : Mm1;
      glds16(cin + r * ldc + c_cc1, base + C::A_BYTES + (2 * wave + 1) * 1024);
    }
    if constexpr (HM) {
      // this wave's 16 keep-mask words of the tile (lanes 0-7, 16 B each)
      const int64_t tt = tile < ntiles ? tile : ntiles - 1;
      if (lane < 8)
        glds16(mask_in + (tt * NT + wave) * 16 + 2 * lane,
               base + C::A_BYTES + C::C_BYTES + wave * 128);
    }
  };

  // ---- prologue: tiles 0 .. NBUF-2 in flight
#pragma unroll
  for (int p = 0; p < NBUF - 1; ++p) issue_tile(t0 + p * G, p);

  // A-fragment read addresses (row col_l of the tile, chunk 2 s + h): with the odd-row
  // swizzle, chunk q lives at q ^ 8, i.e. +-128 B depending on bit 2 of s
  const int r_a = col_l;
  int offP, offM;
  if constexpr (C::RPI == 1) {
    offP = offM = r_a * kPiece + 16 * h;
  } else {
    const int odd = r_a & 1;
    const int base = (r_a >> 1) * kPiece + odd * 512 + 16 * h;
    offP = base + 128 * odd;  // s & 4 == 0: chunk 2s+h has bit 3 clear -> +8 chunks
    offM = base - 128 * odd;  // s & 4 != 0: bit 3 set -> -8 chunks
  }
  const int rsub = 4 * h;
  const int64_t count = (ntiles - 1 - t0) / G + 1;
  int64_t tile = t0;
  for (int64_t i = 0; i < count; ++i, tile += G) {
    const int b = static_cast<int>(i % NBUF);
    // ---- tile i's DMAs done (this wave), then visible to all waves; younger: the DMAs of
    // tiles i+1 .. i+NBUF-2 and the stores of the last min(i, NBUF-1) epilogues
    wait_vmcnt_dyn<(NBUF - 2) * C::OPS, C::STORES_MIN, NBUF - 1>(i);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // ---- refill the buffer every wave finished with (tile i-1's) NBUF-1 tiles ahead;
    // issued unconditionally (past the end: clamped rows, never read) so the counts hold
    issue_tile(tile + (NBUF - 1) * G, static_cast<int>((i + NBUF - 1) % NBUF));

    // ---- MFMA over the staged tile (accumulator starts at the bias: one column per lane)
    const unsigned char* bufp = lds + b * C::BUF;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = bv;
    // A fragments read in groups of FG ahead of their MFMAs (a read issued one MFMA
    // ahead exposed most of the LDS latency at 2 waves / SIMD)
    constexpr int FG = KS > 16 ? 16 : KS;
#pragma unroll
    for (int s0 = 0; s0 < KS; s0 += FG) {
      uint4 af[FG];
#pragma unroll
      for (int u = 0; u < FG; ++u) {
        const int s = s0 + u;
        af[u] = *reinterpret_cast<const uint4*>(bufp + ((s & 4) ? offM : offP) + 32 * s);
      }
#pragma unroll
      for (int u = 0; u < FG; ++u)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8_bs(af[u]), bfr[s0 + u], acc,
                                                      0, 0, 0);
    }

    // ---- epilogue of this tile (this wave's 32x32 output block). Register r of lane l is
    // element (row (r&3) + 8(r>>2) + 4(l>>5), column l&31): the keep bits of register r
    // over the wave ARE a 64-bit lane mask (= tile32 word r), so the ReLU ballot is the
    // compare's own VCC and the input mask is applied as a lane-mask select.
    const int64_t row0 = tile * kTR;
    const int64_t rb = tile;  // 32-row block index (tile32 mask layout)
    const uint16_t* sC = reinterpret_cast<const uint16_t*>(bufp + C::A_BYTES);
    const uint64_t* sM = reinterpret_cast<const uint64_t*>(bufp + C::A_BYTES + C::C_BYTES +
                                                           wave * 128);
    uint32_t wlo = 0, whi = 0;  // lane r < 16: mask word r
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = (r & 3) + 8 * (r >> 2) + rsub;
      float v = acc[r];
      if constexpr (HC) v += bf16_to_f32(sC[rr * N + n]);
      if constexpr (HM) {
        const uint64_t w = sM[r];  // same address in every lane: an LDS broadcast
        const uint32_t wl = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(w));
        const uint32_t wh = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(w >> 32));
        const uint32_t myw = lane < 32 ? wl : wh;
        v = ((myw >> (lane & 31)) & 1u) ? v : 0.f;
      }
      if constexpr (RELU) {
        const bool k = v > 0.f;
        const uint64_t bal = __ballot(k);
        // lane r keeps word r (selects, not a branch; an inline-asm v_writelane of the
        // compare's SGPR result produced wrong words: the hazard recognizer does not see
        // into asm)
        wlo = lane == r ? static_cast<uint32_t>(bal) : wlo;
        whi = lane == r ? static_cast<uint32_t>(bal >> 32) : whi;
        v = k ? v : 0.f;
      }
      sE[rr * kEWs + col_l] = f32_to_bf16(v);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS tile is written
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int rr = (lane >> 2) + 16 * q;
      const int64_t row = row0 + rr;
      if (row < M) {
        const uint4 v = *reinterpret_cast<const uint4*>(&sE[rr * kEWs + (lane & 3) * 8]);
        *reinterpret_cast<uint4*>(out + row * ldo + wave * 32 + (lane & 3) * 8) = v;
      }
    }
    if constexpr (RELU)
      if (mask_out && lane < 16) {
        // word r = lane: lanes 0-31 hold row (r&3) + 8(r>>2), lanes 32-63 that row + 4;
        // rows past M keep nothing
        const int64_t ra = row0 + (lane & 3) + 8 * (lane >> 2);
        const uint32_t lo = ra < M ? wlo : 0u, hi = ra + 4 < M ? whi : 0u;
        mask_out[(rb * NT + wave) * 16 + lane] =
            (static_cast<uint64_t>(hi) << 32) | static_cast<uint64_t>(lo);
      }
  }
  // drain the DMAs issued past the end before the block exits (LDS is released)
  wait_vmcnt<0>();
}

template <int NT, int K, bool HC, bool HM, bool RELU>
hipError_t launch_bs(const void* A1, int64_t lda1, int K1, const void* B1t, const void* A2,
                     int64_t lda2, const void* B2t, const float* bias, const void* cin,
                     int64_t ldc, void* out, int64_t ldo, uint64_t* mask_out,
                     const uint64_t* mask_in, int64_t M, hipStream_t st) {
  using C = BsCfg<NT, K, HC, HM>;
  constexpr size_t lds = C::LDS;
  static_assert(lds <= kLdsMax, "LDS budget");
  auto kern = &dual_gemm_bs_kernel<NT, K, HC, HM, RELU>;
  static int blocks_per_cu = 0;
  static int num_cus = 0;
  if (blocks_per_cu == 0) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        num_cus <= 0)
      num_cus = 256;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(kern),
                                                     NT * 64, lds) != hipSuccess || occ <= 0)
      occ = 1;
    blocks_per_cu = occ > 4 ? 4 : occ;
  }
  const int64_t tiles = (M + kTR - 1) / kTR;
  int64_t blocks = static_cast<int64_t>(num_cus) * blocks_per_cu;
  if (blocks > tiles) blocks = tiles;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(blocks)), dim3(NT * 64), lds, st,
                     static_cast<const uint16_t*>(A1), lda1, K1,
                     static_cast<const uint16_t*>(B1t), static_cast<const uint16_t*>(A2), lda2,
                     static_cast<const uint16_t*>(B2t), bias, static_cast<const uint16_t*>(cin),
                     ldc, static_cast<uint16_t*>(out), ldo, mask_out, mask_in, M);
  return hipGetLastError();
}

template <int NT, int K>
hipError_t bs_by_flags(const void* A1, int64_t lda1, int K1, const void* B1t, const void* A2,
                       int64_t lda2, const void* B2t, const float* bias, const void* cin,
                       int64_t ldc, void* out, int64_t ldo, uint64_t* mo, const uint64_t* mi,
                       int64_t M, bool relu, hipStream_t st) {
#define DG_BS(HC_, HM_)                                                                      \
  if (relu)                                                                                 \
    return launch_bs<NT, K, HC_, HM_, true>(A1, lda1, K1, B1t, A2, lda2, B2t, bias, cin, ldc, \
                                            out, ldo, mo, mi, M, st);                       \
  return launch_bs<NT, K, HC_, HM_, false>(A1, lda1, K1, B1t, A2, lda2, B2t, bias, cin, ldc,  \
                                           out, ldo, mo, mi, M, st);
  if (cin) {
    if (mi) { DG_BS(true, true) }
    DG_BS(true, false)
  }
  if (mi) { DG_BS(false, true) }
  DG_BS(false, false)
#undef DG_BS
}

template <int NT>
hipError_t bs_by_k(int K, const void* A1, int64_t lda1, int K1, const void* B1t,
                   const void* A2, int64_t lda2, const void* B2t, const float* bias,
                   const void* cin, int64_t ldc, void* out, int64_t ldo, uint64_t* mo,
                   const uint64_t* mi, int64_t M, bool relu, hipStream_t st) {
  switch (K) {
    case 192: return bs_by_flags<NT, 192>(A1, lda1, K1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mo, mi, M, relu, st);
    case 256: return bs_by_flags<NT, 256>(A1, lda1, K1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mo, mi, M, relu, st);
    case 512: return bs_by_flags<NT, 512>(A1, lda1, K1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mo, mi, M, relu, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

bool dual_gemm_bs_supported(int64_t N, int64_t K1, int64_t K2) {
  const int64_t K = K1 + K2;
  return dual_gemm_supported(N, K1, K2) && (K == 192 || K == 256 || K == 512);
}

hipError_t dual_gemm_bs(const void* A1, int64_t lda1, const void* B1t, int64_t K1,
                        const void* A2, int64_t lda2, const void* B2t, int64_t K2,
                        const float* bias, const void* cin, int64_t ldc, void* out, int64_t ldo,
                        int64_t M, int64_t N, uint64_t* mask_out, const uint64_t* mask_in,
                        bool relu, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (!dual_gemm_bs_supported(N, K1, K2)) return hipErrorInvalidValue;
  const int K = static_cast<int>(K1 + K2), k1 = static_cast<int>(K1);
  switch (N) {
    case 128: return bs_by_k<4>(K, A1, lda1, k1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mask_out, mask_in, M, relu, st);
    case 192: return bs_by_k<6>(K, A1, lda1, k1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mask_out, mask_in, M, relu, st);
    default: return bs_by_k<8>(K, A1, lda1, k1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mask_out, mask_in, M, relu, st);
  }
}

}  // namespace dgraph
