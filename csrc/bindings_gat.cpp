// dgraph_amd — dispatcher registration of the fused fp32 graph-attention kernels
// (csrc/kernels/gat_f32.hip; models/rgat.py's lean relation layer). Every shape, dtype,
// stride and alignment contract the kernels rely on is checked here; column ids are checked
// against the operand rows once per pattern by the Python caller (ops/gat.py).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "check.h"
#include "kernels/kernels.h"

namespace dgraph {
namespace {

hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

const at::Tensor* opt_t(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? &*t : nullptr;
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

void rows_f32(const at::Tensor& t, const at::Tensor& ref, int64_t min_rows, int64_t cols,
              const char* name) {
  TORCH_CHECK(t.is_cuda() && t.device() == ref.device(), "gat: ", name, " must be on ",
              ref.device());
  TORCH_CHECK(t.scalar_type() == at::kFloat && t.dim() == 2 && t.stride(1) == 1,
              "gat: ", name, " must be 2-D float32 with unit column stride");
  TORCH_CHECK(t.size(0) >= min_rows && t.size(1) == cols, "gat: ", name, " must be at least [",
              min_rows, ", ", cols, "], got ", t.sizes());
  TORCH_CHECK(cols % 4 != 0 || (al16(t.data_ptr()) && t.stride(0) % 4 == 0), "gat: ", name,
              " must be 16-B aligned with a row stride divisible by 4");
}

// per-head score / statistics arrays: [rows, heads] with unit column stride and the row
// stride `lds` shared by every such array of a call (heads for whole rows; a one-head column
// pass hands in column slices of [rows, H] arrays, row stride H)
void scores(const at::Tensor& t, const at::Tensor& ref, int64_t min_rows, int64_t heads,
            int64_t lds, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.device() == ref.device() && t.scalar_type() == at::kFloat &&
                  t.dim() == 2 && t.size(1) == heads && t.size(0) >= min_rows &&
                  (t.size(1) == 1 || t.stride(1) == 1) && t.stride(0) == lds && lds >= heads,
              "gat: ", name, " must be float32 [>= ", min_rows, ", ", heads,
              "] with unit column stride and row stride ", lds, ", got ", t.sizes(), " / ",
              t.strides());
}

IType pattern(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& ref) {
  TORCH_CHECK(rowptr.is_cuda() && rowptr.device() == ref.device() &&
                  rowptr.scalar_type() == at::kLong && rowptr.is_contiguous() &&
                  rowptr.dim() == 1 && rowptr.numel() >= 1,
              "gat: rowptr must be contiguous int64 on ", ref.device());
  TORCH_CHECK(col.is_cuda() && col.device() == ref.device() && col.is_contiguous() &&
                  (col.scalar_type() == at::kInt || col.scalar_type() == at::kLong),
              "gat: col must be contiguous int32/int64 on ", ref.device());
  return col.scalar_type() == at::kInt ? IType::I32 : IType::I64;
}

// sd/out rows = CSR rows; x (+ x2 past nsplit) = the gathered rows
void gat_fwd_op(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& x,
                const c10::optional<at::Tensor>& x2, int64_t nsplit, const at::Tensor& ss,
                const c10::optional<at::Tensor>& ss2, const at::Tensor& sd, at::Tensor& out,
                double beta, at::Tensor& stat_m, at::Tensor& stat_l, int64_t heads,
                double slope) {
  const c10::DeviceGuard guard(x.device());
  const IType it = pattern(rowptr, col, x);
  const int64_t R = rowptr.numel() - 1;
  const int C = static_cast<int>(x.size(1));
  TORCH_CHECK(gat_f32_shape_ok(C, static_cast<int>(heads)), "gat: unsupported width ", C,
              " / heads ", heads, " (C in 64/128/256, >= 2 lanes per head)");
  const int64_t lds = ss.stride(0);
  rows_f32(x, x, 1, C, "x");
  const at::Tensor* p2 = opt_t(x2);
  const at::Tensor* q2 = opt_t(ss2);
  TORCH_CHECK((p2 == nullptr) == (q2 == nullptr), "gat: x2 and ss2 come together");
  TORCH_CHECK(nsplit >= 0 && nsplit < (int64_t(1) << 32), "gat: bad nsplit");
  if (p2) {
    rows_f32(*p2, x, 0, C, "x2");
    scores(*q2, x, p2->size(0), heads, lds, "ss2");
    TORCH_CHECK(x.size(0) >= nsplit, "gat: x has fewer rows than nsplit");
  }
  scores(ss, x, p2 ? nsplit : x.size(0), heads, lds, "ss");
  scores(sd, x, R, heads, lds, "sd");
  rows_f32(out, x, R, C, "out");
  scores(stat_m, x, R, heads, lds, "stat_m");
  scores(stat_l, x, R, heads, lds, "stat_l");
  DG_HIP_CHECK(gat_fwd_f32(it, rowptr.data_ptr<int64_t>(), col.data_ptr(), R, C,
                           static_cast<int>(heads), lds, static_cast<float>(slope),
                           x.data_ptr<float>(), x.stride(0), p2 ? p2->data_ptr<float>() : nullptr,
                           p2 ? p2->stride(0) : 0, p2 ? nsplit : 0, ss.data_ptr<float>(),
                           q2 ? q2->data_ptr<float>() : nullptr, sd.data_ptr<float>(),
                           out.data_ptr<float>(), out.stride(0), static_cast<float>(beta),
                           stat_m.data_ptr<float>(), stat_l.data_ptr<float>(),
                           cur_stream(x)));
}

void gat_bwd_dst_op(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& x,
                    const c10::optional<at::Tensor>& x2, int64_t nsplit, const at::Tensor& ss,
                    const c10::optional<at::Tensor>& ss2, const at::Tensor& sd,
                    const at::Tensor& stat_m, const at::Tensor& stat_l, const at::Tensor& g,
                    at::Tensor& c_out, at::Tensor& gsd_out, int64_t heads, double slope) {
  const c10::DeviceGuard guard(x.device());
  const IType it = pattern(rowptr, col, x);
  const int64_t R = rowptr.numel() - 1;
  const int C = static_cast<int>(x.size(1));
  TORCH_CHECK(gat_f32_shape_ok(C, static_cast<int>(heads)), "gat: unsupported width / heads");
  const int64_t lds = ss.stride(0);
  rows_f32(x, x, 1, C, "x");
  const at::Tensor* p2 = opt_t(x2);
  const at::Tensor* q2 = opt_t(ss2);
  TORCH_CHECK((p2 == nullptr) == (q2 == nullptr), "gat: x2 and ss2 come together");
  TORCH_CHECK(nsplit >= 0 && nsplit < (int64_t(1) << 32), "gat: bad nsplit");
  if (p2) {
    rows_f32(*p2, x, 0, C, "x2");
    scores(*q2, x, p2->size(0), heads, lds, "ss2");
    TORCH_CHECK(x.size(0) >= nsplit, "gat: x has fewer rows than nsplit");
  }
  scores(ss, x, p2 ? nsplit : x.size(0), heads, lds, "ss");
  scores(sd, x, std::max<int64_t>(R, 1), heads, lds, "sd");
  scores(stat_m, x, std::max<int64_t>(R, 1), heads, lds, "stat_m");
  scores(stat_l, x, std::max<int64_t>(R, 1), heads, lds, "stat_l");
  rows_f32(g, x, std::max<int64_t>(R, 1), C, "g");
  scores(c_out, x, R, heads, lds, "c_out");
  scores(gsd_out, x, R, heads, lds, "gsd_out");
  DG_HIP_CHECK(gat_bwd_dst_f32(it, rowptr.data_ptr<int64_t>(), col.data_ptr(), R, C,
                               static_cast<int>(heads), lds, static_cast<float>(slope),
                               x.data_ptr<float>(), x.stride(0),
                               p2 ? p2->data_ptr<float>() : nullptr, p2 ? p2->stride(0) : 0,
                               p2 ? nsplit : 0, ss.data_ptr<float>(),
                               q2 ? q2->data_ptr<float>() : nullptr, sd.data_ptr<float>(),
                               stat_m.data_ptr<float>(), stat_l.data_ptr<float>(),
                               g.data_ptr<float>(), g.stride(0), c_out.data_ptr<float>(),
                               gsd_out.data_ptr<float>(), cur_stream(x)));
}

// rows = source rows (the transposed pattern); col = destination rows
void gat_bwd_src_op(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& g,
                    const at::Tensor& z, const at::Tensor& ss_row, const at::Tensor& sd,
                    const at::Tensor& m_dst, const at::Tensor& l_dst, const at::Tensor& c_dst,
                    const at::Tensor& a_src, at::Tensor& gz,
                    const c10::optional<at::Tensor>& gss, int64_t heads, double slope) {
  const c10::DeviceGuard guard(g.device());
  const IType it = pattern(rowptr, col, g);
  const int64_t R = rowptr.numel() - 1;
  const int C = static_cast<int>(g.size(1));
  TORCH_CHECK(gat_f32_shape_ok(C, static_cast<int>(heads)), "gat: unsupported width / heads");
  const int64_t lds = ss_row.stride(0);
  const int64_t nd = std::max<int64_t>(g.size(0), 1);
  rows_f32(g, g, 1, C, "g");
  rows_f32(z, g, std::max<int64_t>(R, 1), C, "z");
  scores(ss_row, g, std::max<int64_t>(R, 1), heads, lds, "ss_row");
  scores(sd, g, nd, heads, lds, "sd");
  scores(m_dst, g, nd, heads, lds, "m_dst");
  scores(l_dst, g, nd, heads, lds, "l_dst");
  scores(c_dst, g, nd, heads, lds, "c_dst");
  TORCH_CHECK(a_src.is_cuda() && a_src.device() == g.device() &&
                  a_src.scalar_type() == at::kFloat && a_src.is_contiguous() &&
                  a_src.numel() == C && al16(a_src.data_ptr()),
              "gat: a_src must be contiguous float32 [C], 16-B aligned");
  rows_f32(gz, g, R, C, "gz");
  const at::Tensor* pg = opt_t(gss);
  if (pg) scores(*pg, g, R, heads, lds, "gss");
  DG_HIP_CHECK(gat_bwd_src_f32(it, rowptr.data_ptr<int64_t>(), col.data_ptr(), R, C,
                               static_cast<int>(heads), lds, static_cast<float>(slope),
                               g.data_ptr<float>(), g.stride(0), z.data_ptr<float>(),
                               z.stride(0), ss_row.data_ptr<float>(), sd.data_ptr<float>(),
                               m_dst.data_ptr<float>(), l_dst.data_ptr<float>(),
                               c_dst.data_ptr<float>(), a_src.data_ptr<float>(),
                               gz.data_ptr<float>(), gz.stride(0),
                               pg ? pg->data_ptr<float>() : nullptr, cur_stream(g)));
}

}  // namespace
}  // namespace dgraph

TORCH_LIBRARY_FRAGMENT(dgraph_amd, m) {
  m.def("gat_fwd_f32(Tensor rowptr, Tensor col, Tensor x, Tensor? x2, int nsplit, Tensor ss, "
        "Tensor? ss2, Tensor sd, Tensor(a!) out, float beta, Tensor(b!) stat_m, "
        "Tensor(c!) stat_l, int heads, float slope) -> ()");
  m.def("gat_bwd_dst_f32(Tensor rowptr, Tensor col, Tensor x, Tensor? x2, int nsplit, "
        "Tensor ss, Tensor? ss2, Tensor sd, Tensor stat_m, Tensor stat_l, Tensor g, "
        "Tensor(a!) c_out, Tensor(b!) gsd_out, int heads, float slope) -> ()");
  m.def("gat_bwd_src_f32(Tensor rowptr, Tensor col, Tensor g, Tensor z, Tensor ss_row, "
        "Tensor sd, Tensor m_dst, Tensor l_dst, Tensor c_dst, Tensor a_src, Tensor(a!) gz, "
        "Tensor(b!)? gss, int heads, float slope) -> ()");
}

TORCH_LIBRARY_IMPL(dgraph_amd, CUDA, m) {
  m.impl("gat_fwd_f32", &dgraph::gat_fwd_op);
  m.impl("gat_bwd_dst_f32", &dgraph::gat_bwd_dst_op);
  m.impl("gat_bwd_src_f32", &dgraph::gat_bwd_src_op);
}
