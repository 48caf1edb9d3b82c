// dgraph_amd — host launcher API of the gfx950 kernels.
//
// Launchers take raw device pointers plus the caller's hipStream_t (always the
// PyTorch current stream, never the legacy default stream: the reference's
// launchers ignored the stream they fetched, torch_local_kernels.cu:60,105,159,228).
// They return the launch status; the torch binding layer turns errors into c10::Error.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dgraph {

enum class DType : int { F32 = 0, BF16 = 1 };
enum class IType : int { I32 = 0, I64 = 1 };

// ---------------------------------------------------------------------------
// CSR SpMM / segment reduction (K-new-2).
//   out[r, f] = row_scale[r] * sum_{j in [rowptr[r], rowptr[r+1])}
//                 ew[j, h(f)] * col_scale[col[j]] * x[col[j], f]
//               + beta * out[r, f]
// Any of ew / col_scale / row_scale may be null (== 1). h(f) = f / head_dim.
// Deterministic: one wavefront owns an output row, fixed summation order.
// ---------------------------------------------------------------------------
// Kernel selection (tuning / A-B measurement): variant 1 = per-group index loads,
// 2 = cooperative index load + shuffles (default); xcd: row mapping (0 grid-stride,
// 1 XCD-chunked grid-stride, 2 XCD-chunked in-order (default), 3 in-order); pass_cols:
// bf16 rows wider than this (and a multiple of it) run as column passes (0 = never).
// Negative arguments leave a setting unchanged.
void set_spmm_config(int variant, int xcd, int pass_cols);

hipError_t spmm_csr(DType dt, IType it, const int64_t* rowptr, const void* col,
                    const float* ew, int heads, int head_dim, const float* col_scale,
                    const float* row_scale, const void* x, int64_t ldx, void* out,
                    int64_t ldo, int64_t nrows, int F, float beta, hipStream_t stream,
                    int64_t cap = 0, const int64_t* row_map = nullptr);
// row_map (optional, int64 [nrows]): CSR row r writes output row row_map[r] and reads
// row_scale[row_map[r]] (a row-compacted CSR that skips empty rows).

// fp32 row-group SpMM (spmm_f32.hip): F % 4 == 0, 16-B aligned rows and strides.
// row_ids (nullable): group row i aggregates CSR row row_ids[i] (output row i, or
// row_map[i]); col_map (nullable): column c reads x row col_map[c], < 0 skips the entry.
// row_scale is indexed by the OUTPUT row, col_scale by the row of x read.
bool spmm_f32_rowgroup_ok(int F, int64_t ldx, int64_t ldo, const void* x, const void* out);
hipError_t spmm_f32_rowgroup(IType it, const int64_t* rowptr, const void* col,
                             const float* ew, const float* col_scale, const float* row_scale,
                             const int32_t* col_map, const int64_t* row_ids, const float* x,
                             int64_t ldx, float* out, int64_t ldo, int64_t nrows, int F,
                             float beta, int64_t cap, const int64_t* row_map,
                             hipStream_t st, const float* gate = nullptr, int64_t ldgate = 0,
                             const float* self_add = nullptr, int64_t ld_self = 0,
                             const int32_t* self_map = nullptr, int64_t self_row0 = 0);
// self_add (nullable): output row o also gets self_add[self_map[self_row0 + o]] (skipped
// when < 0) after the row scale / beta and before the gate; gate (nullable, indexed like
// out): the stored value is kept where gate > 0, else 0
//
// The full argument set of the same kernel: rowend (nullable) ends row rr's entries at
// rowend[rr] instead of rowptr[rr + 1]; x2 (nullable): column c >= nsplit reads x2 row
// c - nsplit (two sources in one pass; not with col_map / edge weights / col_scale);
// pass_cols: column-pass width of this call (0 = the process default).
struct SpmmF32Args {
  const int64_t* rowptr = nullptr;
  const int64_t* rowend = nullptr;
  const void* col = nullptr;
  IType it = IType::I32;
  const float* ew = nullptr;
  const float* col_scale = nullptr;
  const float* row_scale = nullptr;
  const int32_t* col_map = nullptr;
  const int64_t* row_ids = nullptr;
  const int64_t* row_map = nullptr;
  const float* x = nullptr;
  int64_t ldx = 0;
  const float* x2 = nullptr;
  int64_t ldx2 = 0;
  int64_t nsplit = 0;
  float* out = nullptr;
  int64_t ldo = 0;
  int64_t nrows = 0;
  int F = 0;
  float beta = 0.f;
  int64_t cap = 0;
  const float* gate = nullptr;
  int64_t ldgate = 0;
  const float* self_add = nullptr;
  int64_t ld_self = 0;
  const int32_t* self_map = nullptr;
  int64_t self_row0 = 0;
  int pass_cols = 0;
  int xcd_remap = 0;  // set by the launcher (set_spmm_f32_xcd)
  // 1-bit ReLU keep mask of the output rows (bit c of row o: keep column c), applied last;
  // [out rows, ld_bits] int32 words; bits_col0 = the column of this pass (launcher)
  const uint32_t* keep_bits = nullptr;
  int64_t ld_bits = 0;
  int bits_col0 = 0;
};
hipError_t spmm_f32_run(const SpmmF32Args& a, hipStream_t st);
void set_spmm_f32_pass_cols(int cols);
// rowgroup: 1 = fp32 row-group kernel (default), 0 = generic kernels; pass_cols: column
// pass width (0 = default 64); negative arguments leave a setting unchanged
void set_spmm_f32_config(int rowgroup, int pass_cols);
void set_spmm_f32_grid(int blocks);   // 0 = uncapped
// XCD-contiguous row ranges (1) or plain in-order blocks (0, default): see spmm_f32.hip
void set_spmm_f32_xcd(int on);

// Hub-row splitting (rows whose degree exceeds `cap` are aggregated in three steps):
//   1. spmm_csr(..., cap): every row sums at most its first `cap` entries;
//   2. spmm_hub_partials: segment i = entries [seg_beg[i], seg_end[i]) of one hub row's tail
//      (<= cap entries each), summed (weights as in spmm_csr, one head) into fp32
//      partials[i, :F];
//   3. spmm_hub_reduce: out[hub_rows[h]] += row_scale * sum of partials[hub_seg_ptr[h] ..
//      hub_seg_ptr[h+1]) in segment order (deterministic; no atomics).
hipError_t spmm_hub_partials(DType dt, IType it, const int64_t* seg_beg,
                             const int64_t* seg_end, const void* col, const float* ew,
                             const float* col_scale, const void* x, int64_t ldx,
                             float* partials, int64_t nseg, int F, hipStream_t stream);
hipError_t spmm_hub_reduce(DType dt, const float* partials, const int64_t* hub_seg_ptr,
                           const int64_t* hub_rows, const float* row_scale, void* out,
                           int64_t ldo, int64_t nhub, int F, hipStream_t stream);

// ---------------------------------------------------------------------------
// Row copy with optional source and destination index (K4/K7/K8 replacement, K-new-1).
//   out[dst(i)] (+)= x[src(i)]   for i in [0, n)
// src/dst null == identity. src(i) < 0 writes zeros; dst(i) < 0 skips the row.
// accumulate uses fp32 atomics and requires an fp32 output.
// ---------------------------------------------------------------------------
hipError_t copy_rows(DType dt, IType it, const void* x, int64_t ldx, const void* src_idx,
                     const void* dst_idx, void* out, int64_t ldo, int64_t n, int F,
                     bool accumulate, hipStream_t stream);

// Masked row gather: out[i] = x[idx[i]] where mask[i] == value, else untouched.
hipError_t masked_gather_rows(DType dt, const void* x, int64_t ldx, const int64_t* idx,
                              const int64_t* mask, int64_t value, void* out, int64_t ldo,
                              int64_t n, int F, hipStream_t stream);

// ---------------------------------------------------------------------------
// Edge softmax over CSR segments (K-new-3), numerically stable (max-subtracted;
// the reference omitted it, RGAT.py:154).
//   alpha[j, h] = exp(s[j,h] - max_seg) / sum_seg exp(.)
// backward: ds[j,h] = alpha[j,h] * (g[j,h] - sum_seg alpha*g)
// Scores are fp32 [E, H] in CSR edge order.
// ---------------------------------------------------------------------------
hipError_t edge_softmax_fwd(const int64_t* rowptr, const float* s, float* alpha,
                            int64_t nrows, int H, hipStream_t stream);
hipError_t edge_softmax_bwd(const int64_t* rowptr, const float* alpha, const float* g,
                            float* ds, int64_t nrows, int H, hipStream_t stream);

// ---------------------------------------------------------------------------
// Fused epilogues (elementwise.hip). numel and F must be multiples of 8.
//   bias_relu_pack: y = act(y + bias) in place; bits (may be null) = keep mask,
//                   ceil(numel/512)*16 32-bit words (layout: see elementwise.hip).
//   relu_mask_bwd : g = bit ? g : 0 in place.
//   col_sum_partial: partial[b, :] = column sums of rows of block b (fp32).
// ---------------------------------------------------------------------------
hipError_t bias_relu_pack(DType dt, void* y, const float* bias, uint32_t* bits, int64_t numel,
                          int F, bool relu, hipStream_t stream);
hipError_t relu_mask_bwd(DType dt, void* g, const uint32_t* bits, int64_t numel,
                         hipStream_t stream);
hipError_t col_sum_partial(DType dt, const void* g, int64_t ld, int64_t L, int F,
                           float* partial, int nblocks, hipStream_t stream);
//   row_scale_cols: out[r, 0:w] = x[r, c0:c0+w] * s[r] (x already offset by c0; w % 8 == 0,
//                   16-B aligned rows).
//   row_scale_colsum: row_scale_cols (bf16) + partial[b, 0:w] (row stride ldp) = fp32
//   column sums of the unscaled x over block b's rows (nblocks blocks, fixed partition)
hipError_t row_scale_colsum(const void* x, int64_t ldx, const float* s, void* out,
                            int64_t ldo, int64_t L, int w, float* partial, int64_t ldp,
                            int nblocks, hipStream_t st);
hipError_t row_scale_cols(DType dt, const void* x, int64_t ldx, const float* s, void* out,
                          int64_t ldo, int64_t L, int w, hipStream_t stream);

// fused bias + activation (act.hip): act 0 identity, 1 SiLU, 2 ReLU; F <= 256 (vector lanes)
hipError_t bias_act_fwd(DType dt, int act, const void* z, int64_t ldz, const float* b, void* y,
                        int64_t ldy, int64_t M, int F, hipStream_t st);
hipError_t bias_act_bwd(DType dt, int act, const void* dy, int64_t lddy, const void* z,
                        int64_t ldz, const float* b, void* dz, int64_t lddz, int64_t M, int F,
                        float* partial, int nblocks, hipStream_t st);

// ---------------------------------------------------------------------------
// Fused edge-MLP kernels (edge_fused.hip, K-new-6). mode 0: out[r] = sum relu(R[r]+X[c]);
// mode 1: out[r] = M[r] * #{c : R[r]+X[c] > 0}; mode 2: out[r] = sum X2[c]*[R[r]+X[c] > 0].
// gather_add_act: out[e] = act(Y[e] + P[src[e]] + Q[dst[e]]) (any of Y/P/Q null), act
// 0 none / 1 relu / 2 silu / 3 leaky-relu(0.2); bwd: out[e] = gin[e] * act'(same pre-activation).
// ---------------------------------------------------------------------------
hipError_t pair_relu(DType dt, IType it, int mode, const int64_t* rowptr, const void* col,
                     const void* rowterm, int64_t ldr, const void* gat, int64_t ldg,
                     const void* gat2, int64_t ldg2, const void* rowmul, int64_t ldm, void* out,
                     int64_t ldo, int64_t nrows, int F, hipStream_t st);
hipError_t gather_add_act(DType dt, bool bwd, const void* Y, int64_t ldy, const void* P,
                          int64_t ldp, const int64_t* src, const void* Q, int64_t ldq,
                          const int64_t* dst, const void* gin, int64_t ldgi, void* out,
                          int64_t ldo, int64_t E, int F, int act, hipStream_t st);

// ---------------------------------------------------------------------------
// Row LayerNorm (layernorm.hip). y = (x - mean) * rstd * gamma + beta (+ res); gamma/beta
// fp32 or both null; mean/rstd fp32 [N]. Backward writes dx and per-block fp32 partials
// partial[b][0][:] = sum dy * x_hat, partial[b][1][:] = sum dy (b < nblocks).
// ---------------------------------------------------------------------------
hipError_t layer_norm_fwd(DType dt, const void* x, const float* gamma, const float* beta,
                          const void* res, void* y, float* mean, float* rstd, int64_t N, int F,
                          float eps, hipStream_t st);
hipError_t layer_norm_bwd(DType dt, const void* dy, const void* x, const float* mean,
                          const float* rstd, const float* gamma, void* dx, float* partial,
                          int nblocks, int64_t N, int F, hipStream_t st);

// ---------------------------------------------------------------------------
// Synchronised BatchNorm pieces (batchnorm.hip, K-new-7), fp32 statistics, no fp32 copy
// of x. bn_reduce mode 0: out = (sum (x - center), sum (x - center)^2); mode 1: out =
// (sum dy', sum dy' * xhat), dy' = dy * [xhat*g+b > 0] when relu. out is fp64 [2][F];
// partial is fp32 [nblocks][2][F] scratch with nblocks = bn_reduce_blocks(N).
// bn_apply mode 0: y = act((x - mean) * rstd * g + b); mode 1: dx = (dy' - c1 - xhat * c2)
// * rstd * g. gamma/beta/c1/c2 may be null (g = 1, b = 0).
// ---------------------------------------------------------------------------
int bn_reduce_blocks(int64_t N);
hipError_t bn_reduce(DType dt, int mode, const void* x, int64_t ldx, const void* dy,
                     int64_t ldy, int64_t N, int F, const float* center, const float* rstd,
                     const float* gamma, const float* beta, bool relu, float* partial,
                     int nblocks, double* out, hipStream_t st, float drop_p = 0.f,
                     uint64_t seed = 0);
// drop_p > 0: dropout fused after the activation (forward) / regenerated from (seed,
// element index) on dy (backward, both the reduce and the apply pass)
hipError_t bn_apply(DType dt, int mode, const void* x, int64_t ldx, const void* dy,
                    int64_t ldy, void* out, int64_t ldo, int64_t N, int F, const float* mean,
                    const float* rstd, const float* gamma, const float* beta, const float* c1,
                    const float* c2, bool relu, hipStream_t st, float drop_p = 0.f,
                    uint64_t seed = 0);

// ---------------------------------------------------------------------------
// Fused tall-skinny MFMA dual GEMM (dual_gemm.hip), bf16 in / fp32 accumulate:
//   out = epi(A1 @ B1 (+ A2 @ B2) (+ bias) (+ cin)); B given transposed (Bt[N][K]).
// N in {128,192,256}; K1, K2 in {128,192,256} (K2 = 0: single GEMM); lda % 8 == 0.
// relu: writes keep bits to mask_out ("tile32" layout, see dual_gemm.hip);
// mask_in: zeroes elements whose keep bit is 0. Mask arrays hold
// ceil(M/256) * 8 * (N/32) * 16 uint64 words.
// ---------------------------------------------------------------------------
bool dual_gemm_supported(int64_t N, int64_t K1, int64_t K2);
hipError_t dual_gemm(const void* A1, int64_t lda1, const void* B1t, int64_t K1, const void* A2,
                     int64_t lda2, const void* B2t, int64_t K2, const float* bias,
                     const void* cin, int64_t ldc, void* out, int64_t ldo, int64_t M, int64_t N,
                     uint64_t* mask_out, const uint64_t* mask_in, bool relu, hipStream_t st);
// B-stationary variant (dual_gemm_bs.hip): same contract; A read from HBM once.
// Supports K1 + K2 in {192, 256, 512}; other shapes run the column-half kernel.
bool dual_gemm_bs_supported(int64_t N, int64_t K1, int64_t K2);
hipError_t dual_gemm_bs(const void* A1, int64_t lda1, const void* B1t, int64_t K1,
                        const void* A2, int64_t lda2, const void* B2t, int64_t K2,
                        const float* bias, const void* cin, int64_t ldc, void* out, int64_t ldo,
                        int64_t M, int64_t N, uint64_t* mask_out, const uint64_t* mask_in,
                        bool relu, hipStream_t st);
// ---------------------------------------------------------------------------
// fp32 MFMA dual GEMM (gemm_f32.hip), exact f32 (v_mfma_f32_16x16x4_f32):
//   out[o(i)] = relu?(gate?(A1[a(i)] @ B1 (+ A2[i] @ B2) + bias + beta * cin[o(i)]))
// B row-major [K, N]; N in {64,128,176,192,256}; K1, K2 multiples of 32; 16-B aligned
// operands with leading dimensions % 4 == 0. a_rows / o_rows nullable int64 [M].
// gate (nullable, [*, N] with ldg): v = gate[o(i)][n] > 0 ? v : 0. cin may alias out.
// Work counters of the dynamically scheduled persistent kernels (gemm_f32, wgrad_f32):
// the counter pair {work, blocks done} of stream `st` (one slot per stream, allocated once
// per device; zero at every launch boundary on that stream). Blocks pull tiles / row units
// from it, so a block that cannot start (its CU held by another stream's kernel, e.g.
// RCCL's during a halo exchange) costs nothing: the running blocks take its work. The
// kernel's last block to finish resets the pair (work_counter_release), so no memset is
// enqueued per launch and kernels of different streams never share a slot (launches on
// one stream serialise). A launch recorded into a HIP graph gets a slot of its own (a
// replay may run on any stream, next to eager kernels of the capturing stream), zeroed
// again by its last block for the next replay.
int* work_counter(hipStream_t st);
// Allocate the counter slots of the current device now (before any stream capture).
hipError_t work_counters_init();
// dynamic (work counter, default) or static (block b: tiles b, b + grid, ...) schedule of
// the fp32 GEMM and weight-gradient kernels launched from now on
extern bool g_f32_dynamic;
void set_f32_dynamic(bool on);
// gemm_f32's fused halo pack: output row i is also stored to send rows
// send_pos[send_ptr[i] .. send_ptr[i + 1]) of ``out`` (row stride ``ld``) — applies to the
// next gemm_f32 call only (the binding sets and clears it around that call)
struct GemmSend {
  float* out = nullptr;
  int64_t ld = 0;
  const int64_t* ptr = nullptr;
  const int32_t* pos = nullptr;
};
void set_gemm_f32_send(const GemmSend& s);
bool gemm_f32_supported(int64_t N, int64_t K1, int64_t K2);
hipError_t gemm_f32(const float* A1, int64_t lda1, int64_t K1, const float* B1, int64_t ldb1,
                    const float* A2, int64_t lda2, int64_t K2, const float* B2, int64_t ldb2,
                    const int64_t* a_rows, const float* bias, const float* cin, int64_t ldc,
                    float beta, const float* gate, int64_t ldg, const int64_t* o_rows,
                    const float* row_scale, bool relu, float* out, int64_t ldo, int64_t M,
                    int64_t N, hipStream_t st);
// (row_scale nullable, [M]: the product of row i is scaled by row_scale[i] before bias)
// fp32 weight gradient (wgrad_f32.hip): partials[b] (=|+=) block b's share of
// [A1[a1(m)] | A2[m]]^T G over rows m < M (P blocks, K1 + K2 in {128, 256}, N in
// {128, 176, 192, 256}); wgrad_f32_reduce: out[K*N] = sum_b partials[b] in block order.
bool wgrad_f32_supported(int64_t K, int64_t N);
hipError_t wgrad_f32(const float* A1, int64_t lda1, int64_t K1, const float* A2, int64_t lda2,
                     int64_t K2, const int64_t* a1_rows, const float* G, int64_t ldg,
                     int64_t M, int64_t N, float* partials, int P, int fresh_from,
                     float* col_partials, hipStream_t st);
// (P row units, slab u = unit u, run by min(P, CUs) blocks pulling units dynamically; unit
// u adds into slab u when u < fresh_from, else overwrites it; col_partials (nullable,
// [P, N]): unit u's column sums of G, same accumulate rule — a bias gradient)
hipError_t wgrad_f32_reduce(const float* partials, int P, int64_t KN, float* out,
                            hipStream_t st);
// 1-bit ReLU keep masks of selected rows (bits.hip): F % 32 == 0, F/32 words per row.
hipError_t row_keep_bits(const float* h, int64_t ldh, const int64_t* rows, int64_t n, int F,
                         uint32_t* bits, hipStream_t st);
// rows (nullable): apply to rows rows[0..n) of g (bits indexed by the same row) only
hipError_t apply_keep_bits(float* g, int64_t ldg, const uint32_t* bits, int64_t n, int F,
                           hipStream_t st, const int64_t* rows = nullptr);

// Softmax cross-entropy / argmax of selected logit rows (loss.hip), C <= 256:
//   row_loss[i] = lse(z[rows[i]]) - z[rows[i]][y[i]];  dz[i][c] = (p_c - [c == y]) * scale
//   for c < C and 0 for C <= c < dz_width;  hit[i] = (argmax z[rows[i]] == y[i])
hipError_t xent_rows(const float* z, int64_t ldz, int C, const int64_t* rows, const int64_t* y,
                     int64_t n, float scale, float* dz, int64_t ldd, int dz_width,
                     float* row_loss, hipStream_t st);
hipError_t argmax_hits(const float* z, int64_t ldz, int C, const int64_t* rows,
                       const int64_t* y, int64_t n, uint8_t* hit, hipStream_t st);

// 1 = column-half kernel (dual_gemm.hip), 2 = B-stationary (default); < 0 restores it
void set_dual_gemm_variant(int variant);
int get_dual_gemm_variant();

// ---------------------------------------------------------------------------
// Fused fp32 graph attention of one relation (gat_f32.hip): softmax over each destination
// row's edges of leaky_relu(sd[i] + ss[j]) per head, the weighted gather, and the exact
// adjoint (destination side: c and dL/dsd; source side over the transposed pattern: dz and
// dL/dss). Two sources: columns >= nsplit read x2 / ss2.
bool gat_f32_shape_ok(int C, int heads);
hipError_t gat_fwd_f32(IType it, const int64_t* rowptr, const void* col, int64_t nrows, int C,
                       int heads, int64_t lds, float slope, const float* x, int64_t ldx, const float* x2,
                       int64_t ldx2, int64_t nsplit, const float* ss, const float* ss2,
                       const float* sd, float* out, int64_t ldo, float beta, float* stat_m,
                       float* stat_l, hipStream_t st);
hipError_t gat_bwd_dst_f32(IType it, const int64_t* rowptr, const void* col, int64_t nrows,
                           int C, int heads, int64_t lds, float slope, const float* x, int64_t ldx,
                           const float* x2, int64_t ldx2, int64_t nsplit, const float* ss,
                           const float* ss2, const float* sd, const float* stat_m,
                           const float* stat_l, const float* g, int64_t ldg, float* c_out,
                           float* gsd_out, hipStream_t st);
hipError_t gat_bwd_src_f32(IType it, const int64_t* rowptr, const void* col, int64_t nrows,
                           int C, int heads, int64_t lds, float slope, const float* g, int64_t ldg,
                           const float* z, int64_t ldz, const float* ss_row, const float* sd,
                           const float* m_dst, const float* l_dst, const float* c_dst,
                           const float* a_src, float* gz, int64_t ldgz, float* gss,
                           hipStream_t st);

}  // namespace dgraph
