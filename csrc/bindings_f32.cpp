// dgraph_amd — dispatcher registration of the fp32 (reference-precision) kernels:
// row-group SpMM with input-row lists / column maps, MFMA f32 dual GEMM, split-M weight
// gradient, and the 1-bit keep masks of selected rows. A TORCH_LIBRARY_FRAGMENT of the
// dgraph_amd library (csrc/bindings.cpp); every launch goes to the current HIP stream and
// every shape contract is checked here, before a kernel sees a pointer.
#include <algorithm>
#include <mutex>
#include <vector>
#include <set>
#include <tuple>
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "check.h"
#include "kernels/kernels.h"

namespace dgraph {
namespace {

hipStream_t stream_of(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void same_dev(const at::Tensor& t, const at::Tensor& ref, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.device() == ref.device(), "dgraph_amd: ", name,
              " must be a GPU tensor on ", ref.device());
}

const at::Tensor* opt(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? &*t : nullptr;
}

void f32_rows(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.scalar_type() == at::kFloat && t.dim() == 2 && t.stride(1) == 1,
              "dgraph_amd: ", name, " must be a 2-D float32 tensor with unit column stride");
}

const int64_t* idx64(const c10::optional<at::Tensor>& t, const at::Tensor& ref, int64_t n,
                     const char* name) {
  const at::Tensor* p = opt(t);
  if (!p) return nullptr;
  same_dev(*p, ref, name);
  TORCH_CHECK(p->scalar_type() == at::kLong && p->is_contiguous() && p->numel() == n,
              "dgraph_amd: ", name, " must be contiguous int64 with ", n, " entries");
  return p->data_ptr<int64_t>();
}

// ------------------------------------------------------------------------------------
void spmm_f32_ex_op(const at::Tensor& rowptr, const at::Tensor& col,
                    const c10::optional<at::Tensor>& ew, const c10::optional<at::Tensor>& cs,
                    const c10::optional<at::Tensor>& rs, const c10::optional<at::Tensor>& cmap,
                    const c10::optional<at::Tensor>& row_ids, const at::Tensor& x,
                    const at::Tensor& out, double beta, int64_t cap,
                    const c10::optional<at::Tensor>& row_map,
                    const c10::optional<at::Tensor>& gate,
                    const c10::optional<at::Tensor>& self_add,
                    const c10::optional<at::Tensor>& self_map, int64_t self_row0,
                    const c10::optional<at::Tensor>& rowend,
                    const c10::optional<at::Tensor>& x2, int64_t nsplit, int64_t pass_cols,
                    const c10::optional<at::Tensor>& keep_bits) {
  same_dev(rowptr, x, "rowptr");
  same_dev(col, x, "col");
  same_dev(out, x, "out");
  f32_rows(x, "x");
  f32_rows(out, "out");
  TORCH_CHECK(rowptr.scalar_type() == at::kLong && rowptr.is_contiguous(),
              "rowptr must be contiguous int64");
  TORCH_CHECK(col.is_contiguous() && (col.scalar_type() == at::kInt || col.scalar_type() == at::kLong),
              "col must be contiguous int32/int64");
  TORCH_CHECK(x.size(1) == out.size(1), "x/out feature mismatch");
  const at::Tensor* ri = opt(row_ids);
  const at::Tensor* re = opt(rowend);
  // rows of the CSR: rowptr holds one start per row (+ the end sentinel unless rowend is given)
  const int64_t csr_rows = re ? re->numel() : rowptr.numel() - 1;
  if (re) {
    same_dev(*re, x, "rowend");
    TORCH_CHECK(re->scalar_type() == at::kLong && re->is_contiguous() &&
                    rowptr.numel() >= re->numel(),
                "rowend must be contiguous int64 with at most rowptr's entries");
  }
  const int64_t nrows = ri ? ri->numel() : csr_rows;
  const int64_t* rid = idx64(row_ids, x, nrows, "row_ids");
  const int64_t* rmap = idx64(row_map, x, nrows, "row_map");
  if (!rmap) TORCH_CHECK(out.size(0) >= nrows, "out has fewer rows than the CSR rows");
  auto f32opt = [&](const c10::optional<at::Tensor>& t, const char* name) -> const float* {
    const at::Tensor* p = opt(t);
    if (!p) return nullptr;
    same_dev(*p, x, name);
    TORCH_CHECK(p->scalar_type() == at::kFloat && p->is_contiguous(), name,
                " must be contiguous float32");
    return p->data_ptr<float>();
  };
  SpmmF32Args a;
  a.rowptr = rowptr.data_ptr<int64_t>();
  a.rowend = re ? re->data_ptr<int64_t>() : nullptr;
  a.col = col.data_ptr();
  a.it = col.scalar_type() == at::kInt ? IType::I32 : IType::I64;
  a.ew = f32opt(ew, "edge_weight");
  if (a.ew) TORCH_CHECK(ew->numel() == col.numel(), "edge_weight must be [E]");
  a.col_scale = f32opt(cs, "col_scale");
  a.row_scale = f32opt(rs, "row_scale");
  if (const at::Tensor* p = opt(cmap)) {
    same_dev(*p, x, "col_map");
    TORCH_CHECK(p->scalar_type() == at::kInt && p->is_contiguous(),
                "col_map must be contiguous int32");
    a.col_map = p->data_ptr<int32_t>();
  }
  TORCH_CHECK(spmm_f32_rowgroup_ok(static_cast<int>(x.size(1)), x.stride(0), out.stride(0),
                                   x.data_ptr(), out.data_ptr()),
              "spmm_f32_ex: F % 4 == 0 and 16-B aligned rows/strides required");
  if (const at::Tensor* p = opt(x2)) {
    f32_rows(*p, "x2");
    same_dev(*p, x, "x2");
    TORCH_CHECK(p->size(1) == x.size(1) && p->stride(0) % 4 == 0 &&
                    reinterpret_cast<uintptr_t>(p->data_ptr()) % 16 == 0,
                "x2 must be 16-B aligned, as wide as x, row stride % 4 == 0");
    TORCH_CHECK(nsplit >= 0 && nsplit <= x.size(0) && nsplit < (int64_t(1) << 32),
                "nsplit must be in [0, rows of x]");
    TORCH_CHECK(!a.ew && !a.col_scale,
                "x2 (two sources) is not combined with edge weights / col_scale");
    a.x2 = p->data_ptr<float>();
    a.ldx2 = p->stride(0);
    a.nsplit = nsplit;
  }
  if (const at::Tensor* gt = opt(gate)) {
    f32_rows(*gt, "gate");
    same_dev(*gt, x, "gate");
    TORCH_CHECK(gt->size(1) >= x.size(1) && gt->stride(0) % 4 == 0 &&
                    reinterpret_cast<uintptr_t>(gt->data_ptr()) % 16 == 0,
                "gate must be 16-B aligned with row stride % 4 == 0, width >= F");
    if (!rmap) TORCH_CHECK(gt->size(0) >= nrows, "gate has fewer rows than the output");
    a.gate = gt->data_ptr<float>();
    a.ldgate = gt->stride(0);
  }
  if (const at::Tensor* sa = opt(self_add)) {
    f32_rows(*sa, "self_add");
    same_dev(*sa, x, "self_add");
    const at::Tensor* sm = opt(self_map);
    TORCH_CHECK(sm != nullptr, "self_add needs self_map");
    same_dev(*sm, x, "self_map");
    TORCH_CHECK(sm->scalar_type() == at::kInt && sm->is_contiguous(),
                "self_map must be contiguous int32");
    TORCH_CHECK(sa->size(1) >= x.size(1) && sa->stride(0) % 4 == 0 &&
                    reinterpret_cast<uintptr_t>(sa->data_ptr()) % 16 == 0,
                "self_add must be 16-B aligned with row stride % 4 == 0, width >= F");
    const int64_t max_out = rmap ? out.size(0) : nrows;
    TORCH_CHECK(self_row0 >= 0 && self_row0 + max_out <= sm->numel(),
                "self_map too short for self_row0 + output rows");
    a.self_add = sa->data_ptr<float>();
    a.self_map = sm->data_ptr<int32_t>();
    a.ld_self = sa->stride(0);
    a.self_row0 = self_row0;
  }
  a.row_ids = rid;
  a.row_map = rmap;
  a.x = x.data_ptr<float>();
  a.ldx = x.stride(0);
  a.out = out.data_ptr<float>();
  a.ldo = out.stride(0);
  a.nrows = nrows;
  a.F = static_cast<int>(x.size(1));
  a.beta = static_cast<float>(beta);
  a.cap = cap;
  a.pass_cols = static_cast<int>(pass_cols);
  if (const at::Tensor* kb = opt(keep_bits)) {
    same_dev(*kb, x, "keep_bits");
    TORCH_CHECK(kb->scalar_type() == at::kInt && kb->dim() == 2 && kb->stride(1) == 1,
                "keep_bits must be int32 [rows, words] with unit column stride");
    TORCH_CHECK(kb->size(1) * 32 >= x.size(1), "keep_bits narrower than the columns");
    TORCH_CHECK(kb->size(0) >= (rmap ? out.size(0) : nrows),
                "keep_bits has fewer rows than the output rows");
    a.keep_bits = reinterpret_cast<const uint32_t*>(kb->data_ptr<int32_t>());
    a.ld_bits = kb->stride(0);
  }
  c10::DeviceGuard g(x.device());
  DG_HIP_CHECK(spmm_f32_run(a, stream_of(x)));
}

void gemm_f32_op(const at::Tensor& A1, const at::Tensor& B1, const c10::optional<at::Tensor>& A2,
                 const c10::optional<at::Tensor>& B2, const c10::optional<at::Tensor>& a_rows,
                 const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& cin,
                 double beta, const c10::optional<at::Tensor>& gate,
                 const c10::optional<at::Tensor>& o_rows, bool relu, const at::Tensor& out,
                 const c10::optional<at::Tensor>& row_scale,
                 const c10::optional<at::Tensor>& send_out,
                 const c10::optional<at::Tensor>& send_ptr,
                 const c10::optional<at::Tensor>& send_pos) {
  f32_rows(A1, "A1");
  f32_rows(B1, "B1");
  f32_rows(out, "out");
  same_dev(B1, A1, "B1");
  same_dev(out, A1, "out");
  const at::Tensor* ar = opt(a_rows);
  const int64_t M = ar ? ar->numel() : A1.size(0);
  const int64_t N = B1.size(1), K1 = A1.size(1);
  TORCH_CHECK(B1.size(0) == K1, "gemm_f32: A1/B1 inner dimension mismatch");
  TORCH_CHECK(out.size(1) == N, "gemm_f32: out width != N");
  // the kernel keeps operand row indices in 32 bits
  TORCH_CHECK(A1.size(0) <= INT32_MAX && M <= INT32_MAX, "gemm_f32: more than 2^31 rows");
  const int64_t* arp = idx64(a_rows, A1, M, "a_rows");
  const int64_t* orp = idx64(o_rows, A1, M, "o_rows");
  if (!orp) TORCH_CHECK(out.size(0) >= M, "gemm_f32: out has fewer than M rows");
  const at::Tensor *a2 = opt(A2), *b2 = opt(B2);
  TORCH_CHECK((a2 == nullptr) == (b2 == nullptr), "gemm_f32: A2 and B2 go together");
  int64_t K2 = 0;
  if (a2) {
    f32_rows(*a2, "A2");
    f32_rows(*b2, "B2");
    same_dev(*a2, A1, "A2");
    same_dev(*b2, A1, "B2");
    K2 = a2->size(1);
    TORCH_CHECK(b2->size(0) == K2 && b2->size(1) == N, "gemm_f32: A2/B2 shape mismatch");
    TORCH_CHECK(a2->size(0) >= M, "gemm_f32: A2 has fewer than M rows");
  }
  TORCH_CHECK(gemm_f32_supported(N, K1, K2),
              "gemm_f32: unsupported shape N=", N, " K1=", K1, " K2=", K2);
  const float* bp = nullptr;
  if (const at::Tensor* b = opt(bias)) {
    same_dev(*b, A1, "bias");
    TORCH_CHECK(b->scalar_type() == at::kFloat && b->is_contiguous() && b->numel() == N,
                "bias must be contiguous float32 [N]");
    bp = b->data_ptr<float>();
  }
  const float* cp = nullptr;
  int64_t ldc = 0;
  if (const at::Tensor* c = opt(cin)) {
    f32_rows(*c, "cin");
    same_dev(*c, A1, "cin");
    TORCH_CHECK(c->size(1) == N, "cin width != N");
    if (!orp) TORCH_CHECK(c->size(0) >= M, "cin has fewer than M rows");
    cp = c->data_ptr<float>();
    ldc = c->stride(0);
  }
  const float* gp = nullptr;
  int64_t ldg = 0;
  if (const at::Tensor* gt = opt(gate)) {
    f32_rows(*gt, "gate");
    same_dev(*gt, A1, "gate");
    TORCH_CHECK(gt->size(1) >= N, "gate narrower than N");
    if (!orp) TORCH_CHECK(gt->size(0) >= M, "gate has fewer than M rows");
    gp = gt->data_ptr<float>();
    ldg = gt->stride(0);
  }
  const float* rsp = nullptr;
  if (const at::Tensor* rs = opt(row_scale)) {
    same_dev(*rs, A1, "row_scale");
    TORCH_CHECK(rs->scalar_type() == at::kFloat && rs->is_contiguous() && rs->numel() == M,
                "row_scale must be contiguous float32 [M]");
    rsp = rs->data_ptr<float>();
  }
  // fused halo pack: row i of this call also lands at send rows send_pos[send_ptr[i] ..
  // send_ptr[i + 1]) of send_out (positions checked against send_out's rows on the host)
  GemmSend sd;
  if (const at::Tensor* so = opt(send_out)) {
    const at::Tensor *sp = opt(send_ptr), *sq = opt(send_pos);
    TORCH_CHECK(sp && sq, "gemm_f32: send_out needs send_ptr and send_pos");
    TORCH_CHECK(!orp, "gemm_f32: send_out is not combined with o_rows");
    f32_rows(*so, "send_out");
    same_dev(*so, A1, "send_out");
    same_dev(*sp, A1, "send_ptr");
    same_dev(*sq, A1, "send_pos");
    TORCH_CHECK(so->size(1) == N, "send_out width != N");
    TORCH_CHECK(sp->scalar_type() == at::kLong && sp->is_contiguous() && sp->numel() == M + 1,
                "send_ptr must be contiguous int64 [M + 1]");
    TORCH_CHECK(sq->scalar_type() == at::kInt && sq->is_contiguous(),
                "send_pos must be contiguous int32");
    // bounds of the plan (the kernel writes send_out rows send_pos[q] for q in the
    // send_ptr ranges): a static plan, so checked the first time each plan is seen — after
    // that no per-call device reduction, which would synchronise the host with the stream.
    // A plan is identified by its index tensors' STORAGE (weak references: a freed plan's
    // entry expires, so new tensors reusing its address are checked again), view offsets,
    // sizes and version counters (an in-place rewrite is checked again), and send_out's rows.
    {
      struct Seen {
        c10::weak_intrusive_ptr<c10::StorageImpl> sp, sq;
        int64_t sp_off, sp_n, sq_off, sq_n, rows;
        uint32_t sp_ver, sq_ver;
      };
      static std::mutex mu;
      static std::vector<Seen> seen;
      std::lock_guard<std::mutex> lk(mu);
      seen.erase(std::remove_if(seen.begin(), seen.end(),
                                [](const Seen& e) { return e.sp.expired() || e.sq.expired(); }),
                 seen.end());
      const c10::StorageImpl* spi = sp->storage().unsafeGetStorageImpl();
      const c10::StorageImpl* sqi = sq->storage().unsafeGetStorageImpl();
      const uint32_t spv = sp->_version(), sqv = sq->_version();
      bool hit = false;
      for (const Seen& e : seen) {
        if (e.sp.lock().get() == spi && e.sq.lock().get() == sqi &&
            e.sp_off == sp->storage_offset() && e.sp_n == sp->numel() &&
            e.sq_off == sq->storage_offset() && e.sq_n == sq->numel() && e.rows == so->size(0) &&
            e.sp_ver == spv && e.sq_ver == sqv) {
          hit = true;
          break;
        }
      }
      if (!hit) {
        const int64_t q0 = sp->min().item<int64_t>(), q1 = sp->max().item<int64_t>();
        TORCH_CHECK(q0 >= 0 && q1 <= sq->numel(), "send_ptr outside send_pos");
        if (sq->numel() > 0) {
          const int64_t mn = sq->min().item<int32_t>(), mx = sq->max().item<int32_t>();
          TORCH_CHECK(mn >= 0 && mx < so->size(0), "send_pos outside send_out's rows");
        }
        seen.push_back(Seen{sp->storage().getWeakStorageImpl(),
                            sq->storage().getWeakStorageImpl(), sp->storage_offset(),
                            sp->numel(), sq->storage_offset(), sq->numel(), so->size(0), spv,
                            sqv});
      }
    }
    sd.out = so->data_ptr<float>();
    sd.ld = so->stride(0);
    sd.ptr = sp->data_ptr<int64_t>();
    sd.pos = sq->data_ptr<int32_t>();
  }
  c10::DeviceGuard g(A1.device());
  set_gemm_f32_send(sd);
  const hipError_t err = gemm_f32(
      A1.data_ptr<float>(), A1.stride(0), K1, B1.data_ptr<float>(), B1.stride(0),
      a2 ? a2->data_ptr<float>() : nullptr, a2 ? a2->stride(0) : 0, K2,
      b2 ? b2->data_ptr<float>() : nullptr, b2 ? b2->stride(0) : 0, arp, bp, cp, ldc,
      static_cast<float>(beta), gp, ldg, orp, rsp, relu, out.data_ptr<float>(), out.stride(0),
      M, N, stream_of(A1));
  set_gemm_f32_send(GemmSend{});
  DG_HIP_CHECK(err);
}

void wgrad_f32_op(const at::Tensor& A1, const c10::optional<at::Tensor>& A2,
                  const c10::optional<at::Tensor>& a1_rows, const at::Tensor& G,
                  const at::Tensor& partials, int64_t blocks, int64_t fresh_from,
                  const c10::optional<at::Tensor>& col_partials) {
  f32_rows(A1, "A1");
  f32_rows(G, "G");
  same_dev(G, A1, "G");
  same_dev(partials, A1, "partials");
  const int64_t M = G.size(0), N = G.size(1);
  const int64_t* arp = idx64(a1_rows, A1, M, "a1_rows");
  if (!arp) TORCH_CHECK(A1.size(0) >= M, "wgrad_f32: A1 has fewer rows than G");
  const at::Tensor* a2 = opt(A2);
  int64_t K2 = 0;
  if (a2) {
    f32_rows(*a2, "A2");
    same_dev(*a2, A1, "A2");
    TORCH_CHECK(a2->size(0) >= M, "wgrad_f32: A2 has fewer rows than G");
    K2 = a2->size(1);
  }
  const int64_t K = A1.size(1) + K2;
  TORCH_CHECK(wgrad_f32_supported(K, N), "wgrad_f32: unsupported K=", K, " N=", N);
  TORCH_CHECK(partials.scalar_type() == at::kFloat && partials.is_contiguous() &&
                  partials.dim() == 3 && partials.size(1) == K && partials.size(2) == N,
              "partials must be contiguous float32 [P, K, N]");
  TORCH_CHECK(blocks >= 1 && blocks <= partials.size(0) && fresh_from >= 0 &&
                  fresh_from <= partials.size(0),
              "wgrad_f32: 1 <= blocks <= P and 0 <= fresh_from <= P");
  const at::Tensor* cp = opt(col_partials);
  if (cp) {
    same_dev(*cp, A1, "col_partials");
    TORCH_CHECK(cp->scalar_type() == at::kFloat && cp->is_contiguous() && cp->dim() == 2 &&
                    cp->size(0) >= partials.size(0) && cp->size(1) == N,
                "col_partials must be contiguous float32 [>= P, N]");
  }
  c10::DeviceGuard g(A1.device());
  DG_HIP_CHECK(wgrad_f32(A1.data_ptr<float>(), A1.stride(0), A1.size(1),
                         a2 ? a2->data_ptr<float>() : nullptr, a2 ? a2->stride(0) : 0, K2, arp,
                         G.data_ptr<float>(), G.stride(0), M, N, partials.data_ptr<float>(),
                         static_cast<int>(blocks), static_cast<int>(fresh_from),
                         cp ? cp->data_ptr<float>() : nullptr, stream_of(A1)));
}

void wgrad_f32_reduce_op(const at::Tensor& partials, const at::Tensor& out) {
  same_dev(out, partials, "out");
  TORCH_CHECK(partials.scalar_type() == at::kFloat && partials.is_contiguous() &&
                  partials.dim() == 3,
              "partials must be contiguous float32 [P, K, N]");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() &&
                  out.numel() == partials.size(1) * partials.size(2),
              "out must be contiguous float32 [K, N]");
  c10::DeviceGuard g(out.device());
  DG_HIP_CHECK(wgrad_f32_reduce(partials.data_ptr<float>(), static_cast<int>(partials.size(0)),
                                out.numel(), out.data_ptr<float>(), stream_of(out)));
}

void row_keep_bits_op(const at::Tensor& h, const c10::optional<at::Tensor>& rows,
                      const at::Tensor& bits) {
  f32_rows(h, "h");
  same_dev(bits, h, "bits");
  const at::Tensor* r = opt(rows);
  const int64_t n = r ? r->numel() : h.size(0);
  const int64_t* rp = idx64(rows, h, n, "rows");
  const int F = static_cast<int>(h.size(1));
  TORCH_CHECK(F % 32 == 0, "row_keep_bits: F % 32 != 0");
  TORCH_CHECK(bits.scalar_type() == at::kInt && bits.is_contiguous() &&
                  bits.numel() >= n * (F / 32),
              "bits must be contiguous int32 with >= rows * F/32 words");
  c10::DeviceGuard g(h.device());
  DG_HIP_CHECK(row_keep_bits(h.data_ptr<float>(), h.stride(0), rp, n, F,
                             reinterpret_cast<uint32_t*>(bits.data_ptr<int32_t>()), stream_of(h)));
}

void apply_keep_bits_op(const at::Tensor& g, const at::Tensor& bits,
                        const c10::optional<at::Tensor>& rows) {
  f32_rows(g, "g");
  same_dev(bits, g, "bits");
  const int F = static_cast<int>(g.size(1));
  TORCH_CHECK(F % 32 == 0, "apply_keep_bits: F % 32 != 0");
  TORCH_CHECK(bits.scalar_type() == at::kInt && bits.is_contiguous() &&
                  bits.numel() >= g.size(0) * (F / 32),
              "bits must be contiguous int32 with >= rows * F/32 words");
  const at::Tensor* r = opt(rows);
  const int64_t n = r ? r->numel() : g.size(0);
  // (rows index g and bits alike: each must be a row of g, checked by the caller's plan —
  // the executor passes its loss rows' positions in the support, built once)
  const int64_t* rp = idx64(rows, g, n, "rows");
  c10::DeviceGuard dg(g.device());
  DG_HIP_CHECK(apply_keep_bits(g.data_ptr<float>(), g.stride(0),
                               reinterpret_cast<const uint32_t*>(bits.data_ptr<int32_t>()),
                               n, F, stream_of(g), rp));
}

void xent_rows_op(const at::Tensor& z, const at::Tensor& rows, const at::Tensor& y,
                  double scale, const at::Tensor& dz, const at::Tensor& row_loss, int64_t C) {
  f32_rows(z, "z");
  f32_rows(dz, "dz");
  same_dev(rows, z, "rows");
  same_dev(y, z, "y");
  same_dev(dz, z, "dz");
  same_dev(row_loss, z, "row_loss");
  const int64_t n = rows.numel();
  TORCH_CHECK(rows.scalar_type() == at::kLong && rows.is_contiguous() &&
                  y.scalar_type() == at::kLong && y.is_contiguous() && y.numel() == n,
              "rows / y must be contiguous int64 of equal length");
  TORCH_CHECK(C > 0 && C <= 256 && C <= z.size(1) && dz.size(1) >= C && dz.size(1) <= 256 &&
                  dz.size(0) >= n,
              "xent_rows: C <= 256, z and dz at least C wide, dz >= n rows");
  TORCH_CHECK(row_loss.scalar_type() == at::kFloat && row_loss.is_contiguous() &&
                  row_loss.numel() >= n,
              "row_loss must be contiguous float32 with >= n entries");
  c10::DeviceGuard g(z.device());
  DG_HIP_CHECK(xent_rows(z.data_ptr<float>(), z.stride(0), static_cast<int>(C),
                         rows.data_ptr<int64_t>(), y.data_ptr<int64_t>(), n,
                         static_cast<float>(scale), dz.data_ptr<float>(), dz.stride(0),
                         static_cast<int>(dz.size(1)), row_loss.data_ptr<float>(), stream_of(z)));
}

void argmax_hits_op(const at::Tensor& z, const at::Tensor& rows, const at::Tensor& y,
                    const at::Tensor& hit, int64_t C) {
  f32_rows(z, "z");
  same_dev(rows, z, "rows");
  same_dev(y, z, "y");
  same_dev(hit, z, "hit");
  const int64_t n = rows.numel();
  TORCH_CHECK(rows.scalar_type() == at::kLong && rows.is_contiguous() &&
                  y.scalar_type() == at::kLong && y.is_contiguous() && y.numel() == n,
              "rows / y must be contiguous int64 of equal length");
  TORCH_CHECK(hit.scalar_type() == at::kByte && hit.is_contiguous() && hit.numel() >= n,
              "hit must be contiguous uint8 with >= n entries");
  TORCH_CHECK(C > 0 && C <= 256 && C <= z.size(1), "argmax_hits: 0 < C <= 256, C <= width");
  c10::DeviceGuard g(z.device());
  DG_HIP_CHECK(argmax_hits(z.data_ptr<float>(), z.stride(0), static_cast<int>(C),
                           rows.data_ptr<int64_t>(), y.data_ptr<int64_t>(), n,
                           hit.data_ptr<uint8_t>(), stream_of(z)));
}

void set_spmm_f32_config_op(int64_t rowgroup, int64_t pass_cols) {
  set_spmm_f32_config(static_cast<int>(rowgroup), static_cast<int>(pass_cols));
}

void set_f32_sched_op(int64_t spmm_grid, int64_t dynamic, int64_t spmm_xcd) {
  if (spmm_grid >= 0) set_spmm_f32_grid(static_cast<int>(spmm_grid));
  if (spmm_xcd >= 0) set_spmm_f32_xcd(static_cast<int>(spmm_xcd));
  if (dynamic >= 0) set_f32_dynamic(dynamic != 0);
}

void f32_init_op() { DG_HIP_CHECK(work_counters_init()); }

}  // namespace
}  // namespace dgraph

TORCH_LIBRARY_FRAGMENT(dgraph_amd, m) {
  m.def("set_f32_sched(int spmm_grid=-1, int dynamic=-1, int spmm_xcd=-1) -> ()", &dgraph::set_f32_sched_op);
  m.def("f32_init() -> ()", &dgraph::f32_init_op);
  m.def("set_spmm_f32_config(int rowgroup, int pass_cols=-1) -> ()",
        &dgraph::set_spmm_f32_config_op);
  m.def("spmm_f32_ex(Tensor rowptr, Tensor col, Tensor? edge_weight, Tensor? col_scale, "
        "Tensor? row_scale, Tensor? col_map, Tensor? row_ids, Tensor x, Tensor(a!) out, "
        "float beta=0., int cap=0, Tensor? row_map=None, Tensor? gate=None, "
        "Tensor? self_add=None, Tensor? self_map=None, int self_row0=0, Tensor? rowend=None, "
        "Tensor? x2=None, int nsplit=0, int pass_cols=0, Tensor? keep_bits=None) -> ()");
  m.def("gemm_f32(Tensor A1, Tensor B1, Tensor? A2, Tensor? B2, Tensor? a_rows, Tensor? bias, "
        "Tensor? cin, float beta, Tensor? gate, Tensor? o_rows, bool relu, Tensor(a!) out, "
        "Tensor? row_scale=None, Tensor(b!)? send_out=None, Tensor? send_ptr=None, "
        "Tensor? send_pos=None) -> ()");
  m.def("wgrad_f32(Tensor A1, Tensor? A2, Tensor? a1_rows, Tensor G, Tensor(a!) partials, "
        "int blocks, int fresh_from, Tensor(b!)? col_partials=None) -> ()");
  m.def("wgrad_f32_reduce(Tensor partials, Tensor(a!) out) -> ()");
  m.def("row_keep_bits(Tensor h, Tensor? rows, Tensor(a!) bits) -> ()");
  m.def("apply_keep_bits(Tensor(a!) g, Tensor bits, Tensor? rows=None) -> ()");
  m.def("xent_rows(Tensor z, Tensor rows, Tensor y, float scale, Tensor(a!) dz, "
        "Tensor(b!) row_loss, int C) -> ()");
  m.def("argmax_hits(Tensor z, Tensor rows, Tensor y, Tensor(a!) hit, int C) -> ()");
}

TORCH_LIBRARY_IMPL(dgraph_amd, CUDA, m) {
  m.impl("spmm_f32_ex", &dgraph::spmm_f32_ex_op);
  m.impl("gemm_f32", &dgraph::gemm_f32_op);
  m.impl("wgrad_f32", &dgraph::wgrad_f32_op);
  m.impl("wgrad_f32_reduce", &dgraph::wgrad_f32_reduce_op);
  m.impl("row_keep_bits", &dgraph::row_keep_bits_op);
  m.impl("apply_keep_bits", &dgraph::apply_keep_bits_op);
  m.impl("xent_rows", &dgraph::xent_rows_op);
  m.impl("argmax_hits", &dgraph::argmax_hits_op);
}
