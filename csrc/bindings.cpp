// dgraph_amd — TORCH_LIBRARY registration of the native op library.
//
// Replaces the reference's pybind11 module `torch_local`
// (DGraph/distributed/csrc/torch_local_bindings.cpp:20-26). Registering through the
// dispatcher (not pybind) gives schema-checked ops that autograd.Function wrappers
// and torch.compile can see; every launch goes to the PyTorch current HIP stream.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "check.h"
#include "host/plan_check.h"
#include "kernels/kernels.h"

namespace dgraph {
namespace {

hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

DType dtype_of(const at::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return DType::F32;
  if (t.scalar_type() == at::kBFloat16) return DType::BF16;
  TORCH_CHECK(false, "dgraph_amd: unsupported feature dtype ", t.scalar_type(),
              " (expected float32 or bfloat16)");
}

IType itype_of(const at::Tensor& t) {
  if (t.scalar_type() == at::kInt) return IType::I32;
  if (t.scalar_type() == at::kLong) return IType::I64;
  TORCH_CHECK(false, "dgraph_amd: unsupported index dtype ", t.scalar_type());
}

void check_dev(const at::Tensor& t, const at::Tensor& ref, const char* name) {
  TORCH_CHECK(t.is_cuda(), "dgraph_amd: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.device() == ref.device(), "dgraph_amd: ", name, " on wrong device");
}

void check_rows(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2, "dgraph_amd: ", name, " must be 2-D [rows, F]");
  TORCH_CHECK(t.stride(1) == 1 || t.size(1) <= 1, "dgraph_amd: ", name,
              " must have unit feature stride");
}

const float* opt_f32(const c10::optional<at::Tensor>& t, const at::Tensor& ref,
                     const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_dev(*t, ref, name);
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "dgraph_amd: ", name,
              " must be contiguous float32");
  return t->data_ptr<float>();
}

// --------------------------------------------------------------------------------------
void spmm(const at::Tensor& rowptr, const at::Tensor& col, const c10::optional<at::Tensor>& ew,
          const c10::optional<at::Tensor>& col_scale,
          const c10::optional<at::Tensor>& row_scale, const at::Tensor& x,
          const at::Tensor& out, int64_t heads, int64_t head_dim, double beta, int64_t cap,
          const c10::optional<at::Tensor>& row_map) {
  check_dev(x, x, "x");
  check_dev(rowptr, x, "rowptr");
  check_dev(col, x, "col");
  check_dev(out, x, "out");
  check_rows(x, "x");
  check_rows(out, "out");
  TORCH_CHECK(rowptr.scalar_type() == at::kLong && rowptr.is_contiguous(),
              "rowptr must be contiguous int64");
  TORCH_CHECK(col.is_contiguous(), "col must be contiguous");
  TORCH_CHECK(x.scalar_type() == out.scalar_type(), "x/out dtype mismatch");
  TORCH_CHECK(x.size(1) == out.size(1), "x/out feature mismatch");
  const int64_t nrows = rowptr.numel() - 1;
  const int64_t* rmap = nullptr;
  if (row_map.has_value() && row_map->defined()) {
    check_dev(*row_map, x, "row_map");
    TORCH_CHECK(row_map->scalar_type() == at::kLong && row_map->is_contiguous() &&
                    row_map->numel() == nrows,
                "row_map must be contiguous int64 [nrows]");
    rmap = row_map->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(out.size(0) >= nrows, "out has fewer rows than the CSR");
  }
  const float* ewp = opt_f32(ew, x, "edge_weight");
  if (ewp) TORCH_CHECK(ew->numel() == col.numel() * std::max<int64_t>(heads, 1),
                       "edge_weight must be [E, heads]");
  const float* csp = opt_f32(col_scale, x, "col_scale");
  const float* rsp = opt_f32(row_scale, x, "row_scale");
  c10::DeviceGuard g(x.device());
  const int F = static_cast<int>(x.size(1));
  DG_HIP_CHECK(spmm_csr(dtype_of(x), itype_of(col), rowptr.data_ptr<int64_t>(),
                        col.data_ptr(), ewp, static_cast<int>(heads),
                        static_cast<int>(head_dim), csp, rsp, x.data_ptr(), x.stride(0),
                        out.data_ptr(), out.stride(0), nrows, F, static_cast<float>(beta),
                        cur_stream(x), cap, rmap));
}

// hub-row splitting passes (see kernels.h): fp32 partial sums of the hub-row tails, then
// their fixed-order reduction into the output rows
void spmm_hub_partials_op(const at::Tensor& seg_beg, const at::Tensor& seg_end,
                          const at::Tensor& col, const c10::optional<at::Tensor>& ew,
                          const c10::optional<at::Tensor>& col_scale, const at::Tensor& x,
                          const at::Tensor& partials) {
  check_dev(x, x, "x");
  check_dev(seg_beg, x, "seg_beg");
  check_dev(seg_end, x, "seg_end");
  check_dev(col, x, "col");
  check_dev(partials, x, "partials");
  check_rows(x, "x");
  TORCH_CHECK(seg_beg.scalar_type() == at::kLong && seg_end.scalar_type() == at::kLong &&
                  seg_beg.is_contiguous() && seg_end.is_contiguous() &&
                  seg_beg.numel() == seg_end.numel(),
              "seg_beg/seg_end must be contiguous int64 of equal length");
  TORCH_CHECK(partials.scalar_type() == at::kFloat && partials.is_contiguous() &&
                  partials.dim() == 2 && partials.size(0) >= seg_beg.numel() &&
                  partials.size(1) == x.size(1),
              "partials must be contiguous float32 [nseg, F]");
  TORCH_CHECK(col.is_contiguous(), "col must be contiguous");
  const float* ewp = opt_f32(ew, x, "edge_weight");
  if (ewp) TORCH_CHECK(ew->numel() == col.numel(), "edge_weight must be [E] (one head)");
  const float* csp = opt_f32(col_scale, x, "col_scale");
  c10::DeviceGuard g(x.device());
  DG_HIP_CHECK(spmm_hub_partials(dtype_of(x), itype_of(col), seg_beg.data_ptr<int64_t>(),
                                 seg_end.data_ptr<int64_t>(), col.data_ptr(), ewp, csp,
                                 x.data_ptr(), x.stride(0), partials.data_ptr<float>(),
                                 seg_beg.numel(), static_cast<int>(x.size(1)), cur_stream(x)));
}

void spmm_hub_reduce_op(const at::Tensor& partials, const at::Tensor& hub_seg_ptr,
                        const at::Tensor& hub_rows, const c10::optional<at::Tensor>& row_scale,
                        const at::Tensor& out) {
  check_dev(out, out, "out");
  check_dev(partials, out, "partials");
  check_dev(hub_seg_ptr, out, "hub_seg_ptr");
  check_dev(hub_rows, out, "hub_rows");
  check_rows(out, "out");
  TORCH_CHECK(partials.scalar_type() == at::kFloat && partials.is_contiguous() &&
                  partials.dim() == 2 && partials.size(1) == out.size(1),
              "partials must be contiguous float32 [nseg, F]");
  TORCH_CHECK(hub_seg_ptr.scalar_type() == at::kLong && hub_rows.scalar_type() == at::kLong &&
                  hub_seg_ptr.is_contiguous() && hub_rows.is_contiguous() &&
                  hub_seg_ptr.numel() == hub_rows.numel() + 1,
              "hub_seg_ptr [nhub+1] / hub_rows [nhub] must be contiguous int64");
  const float* rsp = opt_f32(row_scale, out, "row_scale");
  c10::DeviceGuard g(out.device());
  DG_HIP_CHECK(spmm_hub_reduce(dtype_of(out), partials.data_ptr<float>(),
                               hub_seg_ptr.data_ptr<int64_t>(), hub_rows.data_ptr<int64_t>(),
                               rsp, out.data_ptr(), out.stride(0), hub_rows.numel(),
                               static_cast<int>(out.size(1)), cur_stream(out)));
}

void copy_rows_op(const at::Tensor& x, const c10::optional<at::Tensor>& src_idx,
                  const c10::optional<at::Tensor>& dst_idx, const at::Tensor& out,
                  bool accumulate) {
  check_dev(x, x, "x");
  check_dev(out, x, "out");
  check_rows(x, "x");
  check_rows(out, "out");
  TORCH_CHECK(x.scalar_type() == out.scalar_type(), "x/out dtype mismatch");
  TORCH_CHECK(x.size(1) == out.size(1), "x/out feature mismatch");
  if (accumulate) TORCH_CHECK(out.scalar_type() == at::kFloat, "accumulate needs fp32 out");
  const void* sp = nullptr;
  const void* dp = nullptr;
  IType it = IType::I64;
  int64_t n = -1;
  bool have_type = false;
  for (auto* opt : {&src_idx, &dst_idx}) {
    if (opt->has_value() && (*opt)->defined()) {
      const at::Tensor& t = **opt;
      check_dev(t, x, "index");
      TORCH_CHECK(t.dim() == 1 && t.is_contiguous(), "index must be contiguous 1-D");
      if (have_type) {
        TORCH_CHECK(itype_of(t) == it, "src/dst index dtypes must match");
        TORCH_CHECK(t.numel() == n, "src/dst index lengths must match");
      }
      it = itype_of(t);
      n = t.numel();
      have_type = true;
    }
  }
  if (src_idx.has_value() && src_idx->defined()) sp = src_idx->data_ptr();
  if (dst_idx.has_value() && dst_idx->defined()) dp = dst_idx->data_ptr();
  if (n < 0) n = x.size(0);
  c10::DeviceGuard g(x.device());
  DG_HIP_CHECK(copy_rows(dtype_of(x), it, x.data_ptr(), x.stride(0), sp, dp, out.data_ptr(),
                         out.stride(0), n, static_cast<int>(x.size(1)), accumulate,
                         cur_stream(x)));
}

void masked_gather_rows_op(const at::Tensor& x, const at::Tensor& idx, const at::Tensor& mask,
                           int64_t value, const at::Tensor& out) {
  check_dev(x, x, "x");
  check_dev(idx, x, "idx");
  check_dev(mask, x, "mask");
  check_dev(out, x, "out");
  check_rows(x, "x");
  check_rows(out, "out");
  TORCH_CHECK(idx.scalar_type() == at::kLong && mask.scalar_type() == at::kLong,
              "idx/mask must be int64");
  TORCH_CHECK(idx.numel() == mask.numel() && out.size(0) >= idx.numel(), "shape mismatch");
  c10::DeviceGuard g(x.device());
  DG_HIP_CHECK(masked_gather_rows(dtype_of(x), x.data_ptr(), x.stride(0),
                                  idx.contiguous().data_ptr<int64_t>(),
                                  mask.contiguous().data_ptr<int64_t>(), value, out.data_ptr(),
                                  out.stride(0), idx.numel(), static_cast<int>(x.size(1)),
                                  cur_stream(x)));
}

void edge_softmax_fwd_op(const at::Tensor& rowptr, const at::Tensor& s,
                         const at::Tensor& alpha) {
  check_dev(s, s, "scores");
  check_dev(rowptr, s, "rowptr");
  check_dev(alpha, s, "alpha");
  TORCH_CHECK(s.scalar_type() == at::kFloat && s.is_contiguous() && alpha.is_contiguous() &&
                  alpha.scalar_type() == at::kFloat,
              "edge softmax operands must be contiguous fp32");
  const int H = s.dim() == 1 ? 1 : static_cast<int>(s.size(1));
  c10::DeviceGuard g(s.device());
  DG_HIP_CHECK(edge_softmax_fwd(rowptr.data_ptr<int64_t>(), s.data_ptr<float>(),
                                alpha.data_ptr<float>(), rowptr.numel() - 1, H,
                                cur_stream(s)));
}

void edge_softmax_bwd_op(const at::Tensor& rowptr, const at::Tensor& alpha,
                         const at::Tensor& grad, const at::Tensor& ds) {
  check_dev(alpha, alpha, "alpha");
  check_dev(rowptr, alpha, "rowptr");
  check_dev(grad, alpha, "grad");
  check_dev(ds, alpha, "ds");
  TORCH_CHECK(alpha.is_contiguous() && grad.is_contiguous() && ds.is_contiguous() &&
                  grad.scalar_type() == at::kFloat,
              "edge softmax operands must be contiguous fp32");
  const int H = alpha.dim() == 1 ? 1 : static_cast<int>(alpha.size(1));
  c10::DeviceGuard g(alpha.device());
  DG_HIP_CHECK(edge_softmax_bwd(rowptr.data_ptr<int64_t>(), alpha.data_ptr<float>(),
                                grad.data_ptr<float>(), ds.data_ptr<float>(),
                                rowptr.numel() - 1, H, cur_stream(alpha)));
}

void bias_relu_pack_op(const at::Tensor& y, const c10::optional<at::Tensor>& bias,
                       const c10::optional<at::Tensor>& bits, bool relu) {
  check_dev(y, y, "y");
  TORCH_CHECK(y.is_contiguous() && y.dim() == 2, "y must be contiguous 2-D");
  const int64_t F = y.size(1);
  TORCH_CHECK(F % 8 == 0, "bias_relu_pack needs F % 8 == 0");
  const float* bp = opt_f32(bias, y, "bias");
  if (bp) TORCH_CHECK(bias->numel() == F, "bias must have F elements");
  uint32_t* bitp = nullptr;
  if (bits.has_value() && bits->defined()) {
    check_dev(*bits, y, "bits");
    TORCH_CHECK(bits->scalar_type() == at::kInt && bits->is_contiguous() &&
                    bits->numel() >= (y.numel() + 511) / 512 * 16,
                "bits must be contiguous int32 with ceil(numel/512)*16 words");
    bitp = reinterpret_cast<uint32_t*>(bits->data_ptr<int32_t>());
  }
  c10::DeviceGuard g(y.device());
  DG_HIP_CHECK(bias_relu_pack(dtype_of(y), y.data_ptr(), bp, bitp, y.numel(),
                              static_cast<int>(F), relu, cur_stream(y)));
}

void relu_mask_bwd_op(const at::Tensor& g, const at::Tensor& bits) {
  check_dev(g, g, "g");
  check_dev(bits, g, "bits");
  TORCH_CHECK(g.is_contiguous() && g.numel() % 8 == 0, "g must be contiguous, numel%8==0");
  TORCH_CHECK(bits.scalar_type() == at::kInt && bits.numel() >= (g.numel() + 511) / 512 * 16,
              "bad bits");
  c10::DeviceGuard gd(g.device());
  DG_HIP_CHECK(relu_mask_bwd(dtype_of(g), g.data_ptr(),
                             reinterpret_cast<const uint32_t*>(bits.data_ptr<int32_t>()),
                             g.numel(), cur_stream(g)));
}

at::Tensor col_sum_op(const at::Tensor& g) {
  check_dev(g, g, "g");
  check_rows(g, "g");
  const int64_t L = g.size(0), F = g.size(1);
  const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(1024, (L + 255) / 256));
  auto partial = at::empty({nb, F}, g.options().dtype(at::kFloat));
  c10::DeviceGuard gd(g.device());
  DG_HIP_CHECK(col_sum_partial(dtype_of(g), g.data_ptr(), g.stride(0), L,
                               static_cast<int>(F), partial.data_ptr<float>(),
                               static_cast<int>(nb), cur_stream(g)));
  return partial.sum(0);
}

// y = act(z + b) (act: 0 identity, 1 SiLU, 2 ReLU); z, y 2-D row-strided, b fp32 [F] or None
void bias_act_op(const at::Tensor& z, const c10::optional<at::Tensor>& b, int64_t act,
                 const at::Tensor& y) {
  check_dev(z, z, "z");
  check_dev(y, z, "y");
  check_rows(z, "z");
  check_rows(y, "y");
  TORCH_CHECK(z.sizes() == y.sizes() && z.scalar_type() == y.scalar_type(), "z / y mismatch");
  const float* bp = opt_f32(b, z, "b");
  if (bp) TORCH_CHECK(b->numel() == z.size(1) && b->is_contiguous(), "b must be [F]");
  c10::DeviceGuard gd(z.device());
  DG_HIP_CHECK(bias_act_fwd(dtype_of(z), static_cast<int>(act), z.data_ptr(), z.stride(0), bp,
                            y.data_ptr(), y.stride(0), z.size(0), static_cast<int>(z.size(1)),
                            cur_stream(z)));
}

// dz = dy * act'(z + b); returns the bias gradient sum_rows dz (fp32, fixed order)
at::Tensor bias_act_bwd_op(const at::Tensor& dy, const at::Tensor& z,
                           const c10::optional<at::Tensor>& b, int64_t act,
                           const at::Tensor& dz) {
  check_dev(dy, z, "dy");
  check_dev(dz, z, "dz");
  check_rows(dy, "dy");
  check_rows(z, "z");
  check_rows(dz, "dz");
  TORCH_CHECK(dy.sizes() == z.sizes() && dz.sizes() == z.sizes(), "shape mismatch");
  TORCH_CHECK(dy.scalar_type() == z.scalar_type() && dz.scalar_type() == z.scalar_type(),
              "dtype mismatch");
  const float* bp = opt_f32(b, z, "b");
  if (bp) TORCH_CHECK(b->numel() == z.size(1) && b->is_contiguous(), "b must be [F]");
  const int64_t L = z.size(0), F = z.size(1);
  const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(1024, (L + 255) / 256));
  auto partial = at::empty({nb, F}, z.options().dtype(at::kFloat));
  c10::DeviceGuard gd(z.device());
  DG_HIP_CHECK(bias_act_bwd(dtype_of(z), static_cast<int>(act), dy.data_ptr(), dy.stride(0),
                            z.data_ptr(), z.stride(0), bp, dz.data_ptr(), dz.stride(0), L,
                            static_cast<int>(F), partial.data_ptr<float>(),
                            static_cast<int>(nb), cur_stream(z)));
  return partial.sum(0);
}

// out[r, :] = x[r, :] * s[r] for a row-strided 2-D x (a column slice of a wider tensor)
void row_scale_cols_op(const at::Tensor& x, const at::Tensor& s, const at::Tensor& out) {
  check_dev(x, x, "x");
  check_dev(x, out, "out");
  check_dev(x, s, "s");
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.sizes() == out.sizes(), "shape mismatch");
  TORCH_CHECK(x.scalar_type() == out.scalar_type(), "dtype mismatch");
  TORCH_CHECK(s.scalar_type() == at::kFloat && s.is_contiguous() && s.numel() == x.size(0),
              "s must be contiguous fp32 [rows]");
  TORCH_CHECK(x.stride(1) == 1 && out.stride(1) == 1, "rows must be unit-stride");
  const int64_t vec = x.scalar_type() == at::kBFloat16 ? 8 : 4;
  TORCH_CHECK(x.size(1) % vec == 0 && x.stride(0) % vec == 0 && out.stride(0) % vec == 0,
              "row_scale_cols needs 16-B vectors (width and row strides)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "row_scale_cols needs 16-B aligned x/out");
  c10::DeviceGuard gd(x.device());
  DG_HIP_CHECK(row_scale_cols(dtype_of(x), x.data_ptr(), x.stride(0), s.data_ptr<float>(),
                              out.data_ptr(), out.stride(0), x.size(0),
                              static_cast<int>(x.size(1)), cur_stream(x)));
}

// row_scale_cols on bf16 + the column sums of the unscaled x into partial[:, 0:w] (a
// column slice of a [nblocks, F] fp32 partials tensor; the caller sums over dim 0)
void row_scale_colsum_op(const at::Tensor& x, const at::Tensor& s, const at::Tensor& out,
                         const at::Tensor& partial) {
  check_dev(x, x, "x");
  check_dev(x, out, "out");
  check_dev(x, s, "s");
  check_dev(x, partial, "partial");
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.sizes() == out.sizes(), "shape mismatch");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16,
              "row_scale_colsum is bf16");
  TORCH_CHECK(s.scalar_type() == at::kFloat && s.is_contiguous() && s.numel() == x.size(0),
              "s must be contiguous fp32 [rows]");
  TORCH_CHECK(x.stride(1) == 1 && out.stride(1) == 1, "rows must be unit-stride");
  TORCH_CHECK(x.size(1) % 8 == 0 && x.size(1) <= 256 && x.stride(0) % 8 == 0 &&
                  out.stride(0) % 8 == 0,
              "row_scale_colsum needs 16-B vectors and width <= 256");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "row_scale_colsum needs 16-B aligned x/out");
  TORCH_CHECK(partial.scalar_type() == at::kFloat && partial.dim() == 2 &&
                  partial.size(1) == x.size(1) && partial.stride(1) == 1 &&
                  partial.size(0) >= 1 && partial.size(0) <= 65535,
              "partial must be fp32 [nblocks, w] with unit column stride");
  c10::DeviceGuard gd(x.device());
  DG_HIP_CHECK(row_scale_colsum(x.data_ptr(), x.stride(0), s.data_ptr<float>(), out.data_ptr(),
                                out.stride(0), x.size(0), static_cast<int>(x.size(1)),
                                partial.data_ptr<float>(), partial.stride(0),
                                static_cast<int>(partial.size(0)), cur_stream(x)));
}

// mode 0 (agg): out[r] = sum_c relu(rowterm[r] + gat[c]); mode 1 (cnt): out[r] = rowmul[r] *
// #{c : rowterm[r] + gat[c] > 0}; mode 2 (tgrad): out[r] = sum_c gat2[c] * [rowterm[r]+gat[c]>0]
void pair_relu_op(const at::Tensor& rowptr, const at::Tensor& col, int64_t mode,
                  const at::Tensor& rowterm, const at::Tensor& gat,
                  const c10::optional<at::Tensor>& gat2, const c10::optional<at::Tensor>& rowmul,
                  const at::Tensor& out) {
  check_dev(rowterm, rowterm, "rowterm");
  for (const at::Tensor* t : {&rowptr, &col, &gat, &out}) check_dev(*t, rowterm, "operand");
  check_rows(rowterm, "rowterm");
  check_rows(gat, "gat");
  check_rows(out, "out");
  TORCH_CHECK(mode >= 0 && mode <= 2, "pair_relu: mode must be 0, 1 or 2");
  TORCH_CHECK(rowptr.scalar_type() == at::kLong && rowptr.is_contiguous() && col.is_contiguous(),
              "rowptr must be contiguous int64, col contiguous");
  const int64_t nrows = rowptr.numel() - 1;
  const int64_t F = out.size(1);
  TORCH_CHECK(rowterm.size(0) >= nrows && out.size(0) >= nrows && rowterm.size(1) == F &&
                  gat.size(1) == F,
              "pair_relu: shape mismatch");
  TORCH_CHECK(rowterm.scalar_type() == gat.scalar_type() &&
                  out.scalar_type() == gat.scalar_type(),
              "pair_relu: dtype mismatch");
  const void* g2 = nullptr;
  int64_t ldg2 = 0;
  if (mode == 2) {
    TORCH_CHECK(gat2.has_value() && gat2->defined(), "pair_relu mode 2 needs gat2");
    check_dev(*gat2, rowterm, "gat2");
    check_rows(*gat2, "gat2");
    TORCH_CHECK(gat2->size(1) == F && gat2->scalar_type() == gat.scalar_type(), "gat2 mismatch");
    g2 = gat2->data_ptr();
    ldg2 = gat2->stride(0);
  }
  const void* m = nullptr;
  int64_t ldm = 0;
  if (mode == 1) {
    TORCH_CHECK(rowmul.has_value() && rowmul->defined(), "pair_relu mode 1 needs rowmul");
    check_dev(*rowmul, rowterm, "rowmul");
    check_rows(*rowmul, "rowmul");
    TORCH_CHECK(rowmul->size(1) == F && rowmul->size(0) >= nrows &&
                    rowmul->scalar_type() == gat.scalar_type(),
                "rowmul mismatch");
    m = rowmul->data_ptr();
    ldm = rowmul->stride(0);
  }
  c10::DeviceGuard g(out.device());
  DG_HIP_CHECK(pair_relu(dtype_of(out), itype_of(col), static_cast<int>(mode),
                         rowptr.data_ptr<int64_t>(), col.data_ptr(), rowterm.data_ptr(),
                         rowterm.stride(0), gat.data_ptr(), gat.stride(0), g2, ldg2, m, ldm,
                         out.data_ptr(), out.stride(0), nrows, static_cast<int>(F),
                         cur_stream(out)));
}

// out[e] = act(Y[e] + P[src[e]] + Q[dst[e]]) ; with gin: out[e] = gin[e] * act'(...)
void gather_add_act_op(const c10::optional<at::Tensor>& Y, const c10::optional<at::Tensor>& P,
                       const c10::optional<at::Tensor>& src, const c10::optional<at::Tensor>& Q,
                       const c10::optional<at::Tensor>& dst, const c10::optional<at::Tensor>& gin,
                       const at::Tensor& out, int64_t act) {
  check_dev(out, out, "out");
  check_rows(out, "out");
  TORCH_CHECK(act >= 0 && act <= 3, "act must be 0 (none), 1 (relu), 2 (silu), 3 (leaky 0.2)");
  const int64_t E = out.size(0), F = out.size(1);
  auto opt_rows = [&](const c10::optional<at::Tensor>& t, const char* name, bool per_edge,
                      int64_t& ld) -> const void* {
    if (!t.has_value() || !t->defined()) return nullptr;
    check_dev(*t, out, name);
    check_rows(*t, name);
    TORCH_CHECK(t->size(1) == F && t->scalar_type() == out.scalar_type(), name, " mismatch");
    if (per_edge) TORCH_CHECK(t->size(0) >= E, name, " has too few rows");
    ld = t->stride(0);
    return t->data_ptr();
  };
  auto opt_idx = [&](const c10::optional<at::Tensor>& t, const char* name) -> const int64_t* {
    TORCH_CHECK(t.has_value() && t->defined(), name, " index required");
    check_dev(*t, out, name);
    TORCH_CHECK(t->scalar_type() == at::kLong && t->is_contiguous() && t->numel() >= E, name,
                " must be contiguous int64 with E entries");
    return t->data_ptr<int64_t>();
  };
  int64_t ldy = 0, ldp = 0, ldq = 0, ldg = 0;
  const void* y = opt_rows(Y, "Y", true, ldy);
  const void* p = opt_rows(P, "P", false, ldp);
  const void* q = opt_rows(Q, "Q", false, ldq);
  const void* gi = opt_rows(gin, "gin", true, ldg);
  const int64_t* sp = p ? opt_idx(src, "src") : nullptr;
  const int64_t* dp = q ? opt_idx(dst, "dst") : nullptr;
  c10::DeviceGuard g(out.device());
  DG_HIP_CHECK(gather_add_act(dtype_of(out), gi != nullptr, y, ldy, p, ldp, sp, q, ldq, dp, gi,
                              ldg, out.data_ptr(), out.stride(0), E, static_cast<int>(F),
                              static_cast<int>(act), cur_stream(out)));
}

bool ln_shape_ok(const at::Tensor& x) {
  const int64_t F = x.size(1);
  const int V = x.scalar_type() == at::kFloat ? 4 : 8;
  const int64_t per = (F % V == 0) ? F / V : F;
  return (per + 63) / 64 <= 8;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> layer_norm_fwd_op(
    const at::Tensor& x, const c10::optional<at::Tensor>& gamma,
    const c10::optional<at::Tensor>& beta, const c10::optional<at::Tensor>& res, double eps) {
  check_dev(x, x, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "layer_norm: x must be contiguous [N, F]");
  TORCH_CHECK(ln_shape_ok(x), "layer_norm: feature width too large for the kernel");
  const int64_t N = x.size(0), F = x.size(1);
  const float* gp = opt_f32(gamma, x, "gamma");
  const float* bp = opt_f32(beta, x, "beta");
  TORCH_CHECK((gp == nullptr) == (bp == nullptr), "gamma and beta must both be given or not");
  if (gp) TORCH_CHECK(gamma->numel() == F && beta->numel() == F, "gamma/beta must have F elems");
  const void* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_dev(*res, x, "res");
    TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous() &&
                    res->scalar_type() == x.scalar_type(),
                "res must match x");
    rp = res->data_ptr();
  }
  auto y = at::empty_like(x);
  auto opts = x.options().dtype(at::kFloat);
  auto mean = at::empty({N}, opts);
  auto rstd = at::empty({N}, opts);
  c10::DeviceGuard g(x.device());
  DG_HIP_CHECK(layer_norm_fwd(dtype_of(x), x.data_ptr(), gp, bp, rp, y.data_ptr(),
                              mean.data_ptr<float>(), rstd.data_ptr<float>(), N,
                              static_cast<int>(F), static_cast<float>(eps), cur_stream(x)));
  return {y, mean, rstd};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> layer_norm_bwd_op(
    const at::Tensor& dy, const at::Tensor& x, const at::Tensor& mean, const at::Tensor& rstd,
    const c10::optional<at::Tensor>& gamma) {
  check_dev(x, x, "x");
  check_dev(dy, x, "dy");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && dy.is_contiguous() &&
                  dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(),
              "layer_norm_bwd: dy/x must be contiguous [N, F] of one dtype");
  TORCH_CHECK(ln_shape_ok(x), "layer_norm: feature width too large for the kernel");
  const int64_t N = x.size(0), F = x.size(1);
  TORCH_CHECK(mean.numel() == N && rstd.numel() == N && mean.scalar_type() == at::kFloat &&
                  rstd.scalar_type() == at::kFloat,
              "mean/rstd must be fp32 [N]");
  const float* gp = opt_f32(gamma, x, "gamma");
  auto dx = at::empty_like(x);
  // 4096 blocks x 4 waves keeps ~16 waves per CU streaming; the [nb, 2, F] fp32 partials
  // (4 MB at F = 128) are summed in a fixed order below
  const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(4096, (N + 255) / 256));
  auto partial = at::empty({nb, 2, F}, x.options().dtype(at::kFloat));
  c10::DeviceGuard g(x.device());
  DG_HIP_CHECK(layer_norm_bwd(dtype_of(x), dy.data_ptr(), x.data_ptr(), mean.data_ptr<float>(),
                              rstd.data_ptr<float>(), gp, dx.data_ptr(), partial.data_ptr<float>(),
                              static_cast<int>(nb), N, static_cast<int>(F), cur_stream(x)));
  auto sums = partial.sum(0);
  return {dx, sums[0], sums[1]};
}

// -------------------------------------------------------------------------------- BN
void bn_check(const at::Tensor& t, const at::Tensor& ref, const char* name) {
  check_dev(t, ref, name);
  check_rows(t, name);
  TORCH_CHECK(t.sizes() == ref.sizes() && t.scalar_type() == ref.scalar_type(), "bn: ", name,
              " must match x");
}

const float* bn_vec(const c10::optional<at::Tensor>& t, const at::Tensor& x, const char* name) {
  const float* p = opt_f32(t, x, name);
  if (p) TORCH_CHECK(t->numel() == x.size(1), "bn: ", name, " must have F elements");
  return p;
}

at::Tensor bn_reduce_op(const at::Tensor& x, const c10::optional<at::Tensor>& dy,
                        const at::Tensor& center, const c10::optional<at::Tensor>& rstd,
                        const c10::optional<at::Tensor>& gamma,
                        const c10::optional<at::Tensor>& beta, bool relu, int64_t mode,
                        double drop_p, int64_t seed) {
  check_dev(x, x, "x");
  check_rows(x, "x");
  TORCH_CHECK(mode == 0 || mode == 1, "bn_reduce: mode 0 (stats) or 1 (backward)");
  const void* dyp = nullptr;
  int64_t ldy = 0;
  if (mode == 1) {
    TORCH_CHECK(dy.has_value() && dy->defined(), "bn_reduce: backward needs dy");
    bn_check(*dy, x, "dy");
    dyp = dy->data_ptr();
    ldy = dy->stride(0);
    TORCH_CHECK(rstd.has_value() && rstd->defined(), "bn_reduce: backward needs rstd");
  }
  const int64_t N = x.size(0), F = x.size(1);
  const int nb = bn_reduce_blocks(N);
  auto partial = at::empty({nb, 2, F}, x.options().dtype(at::kFloat));
  auto out = at::empty({2, F}, x.options().dtype(at::kDouble));
  c10::DeviceGuard g(x.device());
  DG_HIP_CHECK(bn_reduce(dtype_of(x), static_cast<int>(mode), x.data_ptr(), x.stride(0), dyp, ldy,
                         N, static_cast<int>(F), bn_vec(center, x, "center"),
                         bn_vec(rstd, x, "rstd"), bn_vec(gamma, x, "gamma"),
                         bn_vec(beta, x, "beta"), relu, partial.data_ptr<float>(), nb,
                         out.data_ptr<double>(), cur_stream(x), static_cast<float>(drop_p),
                         static_cast<uint64_t>(seed)));
  return out;
}

at::Tensor bn_apply_op(const at::Tensor& x, const c10::optional<at::Tensor>& dy,
                       const at::Tensor& mean, const at::Tensor& rstd,
                       const c10::optional<at::Tensor>& gamma,
                       const c10::optional<at::Tensor>& beta, const c10::optional<at::Tensor>& c1,
                       const c10::optional<at::Tensor>& c2, bool relu, int64_t mode,
                       double drop_p, int64_t seed) {
  check_dev(x, x, "x");
  check_rows(x, "x");
  TORCH_CHECK(mode == 0 || mode == 1, "bn_apply: mode 0 (forward) or 1 (backward)");
  const void* dyp = nullptr;
  int64_t ldy = 0;
  if (mode == 1) {
    TORCH_CHECK(dy.has_value() && dy->defined(), "bn_apply: backward needs dy");
    bn_check(*dy, x, "dy");
    dyp = dy->data_ptr();
    ldy = dy->stride(0);
  }
  auto out = at::empty(x.sizes(), x.options());
  c10::DeviceGuard g(x.device());
  DG_HIP_CHECK(bn_apply(dtype_of(x), static_cast<int>(mode), x.data_ptr(), x.stride(0), dyp, ldy,
                        out.data_ptr(), out.stride(0), x.size(0), static_cast<int>(x.size(1)),
                        bn_vec(mean, x, "mean"), bn_vec(rstd, x, "rstd"),
                        bn_vec(gamma, x, "gamma"), bn_vec(beta, x, "beta"), bn_vec(c1, x, "c1"),
                        bn_vec(c2, x, "c2"), relu, cur_stream(x), static_cast<float>(drop_p),
                        static_cast<uint64_t>(seed)));
  return out;
}

int64_t tile32_mask_words(int64_t M, int64_t N) { return (M + 255) / 256 * 8 * (N / 32) * 16; }

void dual_gemm_op(const at::Tensor& A1, const at::Tensor& B1t, const c10::optional<at::Tensor>& A2,
                  const c10::optional<at::Tensor>& B2t, const c10::optional<at::Tensor>& bias,
                  const c10::optional<at::Tensor>& cin, const at::Tensor& out,
                  const c10::optional<at::Tensor>& mask_out,
                  const c10::optional<at::Tensor>& mask_in, bool relu) {
  auto chk_bf16 = [&](const at::Tensor& t, const char* name) {
    check_dev(t, out, name);
    TORCH_CHECK(t.scalar_type() == at::kBFloat16, "dual_gemm: ", name, " must be bfloat16");
    TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, "dual_gemm: ", name,
                " must be 2-D with unit inner stride");
  };
  chk_bf16(out, "out");
  chk_bf16(A1, "A1");
  chk_bf16(B1t, "B1t");
  const int64_t M = A1.size(0), K1 = A1.size(1), N = B1t.size(0);
  TORCH_CHECK(B1t.size(1) == K1 && B1t.is_contiguous(), "B1t must be contiguous [N, K1]");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N, "out must be [M, N]");
  // the kernel moves A, cin and out rows in 16-B vectors
  auto al16 = [](const at::Tensor& t) {
    return t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0;
  };
  TORCH_CHECK(al16(A1) && al16(out), "dual_gemm: A1/out rows must be 16-B aligned");
  const void* a2 = nullptr;
  const void* b2 = nullptr;
  int64_t K2 = 0, lda2 = 0;
  if (A2.has_value() && A2->defined()) {
    chk_bf16(*A2, "A2");
    TORCH_CHECK(B2t.has_value() && B2t->defined(), "A2 needs B2t");
    chk_bf16(*B2t, "B2t");
    K2 = A2->size(1);
    TORCH_CHECK(A2->size(0) == M && B2t->size(0) == N && B2t->size(1) == K2 &&
                    B2t->is_contiguous() && al16(*A2),
                "A2/B2t shape mismatch");
    a2 = A2->data_ptr();
    b2 = B2t->data_ptr();
    lda2 = A2->stride(0);
  }
  TORCH_CHECK(dual_gemm_supported(N, K1, K2), "dual_gemm: unsupported shape N=", N, " K1=", K1,
              " K2=", K2);
  const float* bp = opt_f32(bias, out, "bias");
  if (bp) TORCH_CHECK(bias->numel() == N, "bias must have N elements");
  const void* cp = nullptr;
  int64_t ldc = 0;
  if (cin.has_value() && cin->defined()) {
    chk_bf16(*cin, "cin");
    TORCH_CHECK(cin->size(0) == M && cin->size(1) == N && al16(*cin),
                "cin must be [M, N] with 16-B aligned rows");
    cp = cin->data_ptr();
    ldc = cin->stride(0);
  }
  auto mask_ptr = [&](const c10::optional<at::Tensor>& m, const char* name) -> void* {
    if (!m.has_value() || !m->defined()) return nullptr;
    check_dev(*m, out, name);
    TORCH_CHECK(m->scalar_type() == at::kLong && m->is_contiguous() &&
                    m->numel() >= tile32_mask_words(M, N),
                name, " must be contiguous int64 with ", tile32_mask_words(M, N), " words");
    return m->data_ptr();
  };
  auto* mo = static_cast<uint64_t*>(mask_ptr(mask_out, "mask_out"));
  auto* mi = static_cast<const uint64_t*>(mask_ptr(mask_in, "mask_in"));
  c10::DeviceGuard g(out.device());
  DG_HIP_CHECK(dual_gemm(A1.data_ptr(), A1.stride(0), B1t.data_ptr(), K1, a2, lda2, b2, K2, bp,
                         cp, ldc, out.data_ptr(), out.stride(0), M, N, mo, mi, relu,
                         cur_stream(out)));
}

}  // namespace
}  // namespace dgraph

int64_t tile32_mask_words_op(int64_t M, int64_t N) { return dgraph::tile32_mask_words(M, N); }

void set_spmm_config_op(int64_t variant, int64_t xcd, int64_t pass_cols) {
  dgraph::set_spmm_config(static_cast<int>(variant), static_cast<int>(xcd),
                          static_cast<int>(pass_cols));
}

void set_dual_gemm_variant_op(int64_t variant) {
  dgraph::set_dual_gemm_variant(static_cast<int>(variant));
}
int64_t get_dual_gemm_variant_op() { return dgraph::get_dual_gemm_variant(); }

// --- host-side plan validation (csrc/host/plan_check.*; DGRAPH_CHECK_PLANS=1) ----------
namespace {
at::Tensor host_i64(const at::Tensor& t) { return t.to(at::kCPU, at::kLong).contiguous(); }

void raise_if_bad(const dgraph::host::CheckResult& r, const char* what) {
  TORCH_CHECK(r.ok, what, ": ", r.what, " (at index ", r.where, ")");
}
}  // namespace

void validate_csr_op(const at::Tensor& rowptr, const at::Tensor& col, int64_t ncols) {
  const at::Tensor rp = host_i64(rowptr);
  TORCH_CHECK(col.scalar_type() == at::kInt || col.scalar_type() == at::kLong,
              "validate_csr: col must be int32 or int64");
  const at::Tensor c = col.to(at::kCPU).contiguous();
  raise_if_bad(dgraph::host::check_csr(rp.data_ptr<int64_t>(), rp.numel() - 1, c.data_ptr(),
                                       static_cast<int>(c.element_size()), c.numel(), ncols),
               "validate_csr");
}

void validate_row_map_op(const at::Tensor& row_map, int64_t nrows_out) {
  const at::Tensor m = host_i64(row_map);
  raise_if_bad(dgraph::host::check_row_map(m.data_ptr<int64_t>(), m.numel(), nrows_out),
               "validate_row_map");
}

void validate_hub_split_op(const at::Tensor& rowptr, const at::Tensor& seg_row,
                           const at::Tensor& seg_lo, const at::Tensor& seg_hi, int64_t head) {
  const at::Tensor rp = host_i64(rowptr), r = host_i64(seg_row), lo = host_i64(seg_lo),
                   hi = host_i64(seg_hi);
  TORCH_CHECK(r.numel() == lo.numel() && r.numel() == hi.numel(), "segment arrays differ");
  raise_if_bad(dgraph::host::check_hub_split(rp.data_ptr<int64_t>(), rp.numel() - 1,
                                             r.data_ptr<int64_t>(), lo.data_ptr<int64_t>(),
                                             hi.data_ptr<int64_t>(), r.numel(), head),
               "validate_hub_split");
}

void validate_splits_op(const at::Tensor& send, const at::Tensor& recv, int64_t total_send,
                        int64_t total_recv) {
  const at::Tensor s = host_i64(send), r = host_i64(recv);
  TORCH_CHECK(s.numel() == r.numel(), "split vectors differ in length");
  raise_if_bad(dgraph::host::check_splits(s.data_ptr<int64_t>(), r.data_ptr<int64_t>(),
                                          static_cast<int>(s.numel()), total_send, total_recv),
               "validate_splits");
}

TORCH_LIBRARY(dgraph_amd, m) {
  m.def("set_dual_gemm_variant(int variant) -> ()", &set_dual_gemm_variant_op);
  m.def("get_dual_gemm_variant() -> int", &get_dual_gemm_variant_op);
  m.def("validate_csr(Tensor rowptr, Tensor col, int ncols) -> ()", &validate_csr_op);
  m.def("validate_row_map(Tensor row_map, int nrows_out) -> ()", &validate_row_map_op);
  m.def("validate_hub_split(Tensor rowptr, Tensor seg_row, Tensor seg_lo, Tensor seg_hi, "
        "int head=0) -> ()",
        &validate_hub_split_op);
  m.def("validate_splits(Tensor send, Tensor recv, int total_send, int total_recv) -> ()",
        &validate_splits_op);
  m.def("set_spmm_config(int variant, int xcd, int pass_cols=-1) -> ()", &set_spmm_config_op);
  m.def("bias_relu_pack(Tensor(a!) y, Tensor? bias, Tensor(b!)? bits, bool relu) -> ()");
  m.def("relu_mask_bwd(Tensor(a!) g, Tensor bits) -> ()");
  m.def("col_sum(Tensor g) -> Tensor");
  m.def("bias_act(Tensor z, Tensor? b, int act, Tensor(a!) y) -> ()");
  m.def("bias_act_bwd(Tensor dy, Tensor z, Tensor? b, int act, Tensor(a!) dz) -> Tensor");
  m.def("row_scale_cols(Tensor x, Tensor s, Tensor(a!) out) -> ()");
  m.def("row_scale_colsum(Tensor x, Tensor s, Tensor(a!) out, Tensor(b!) partial) -> ()");
  m.def("pair_relu(Tensor rowptr, Tensor col, int mode, Tensor rowterm, Tensor gat, Tensor? gat2, "
        "Tensor? rowmul, Tensor(a!) out) -> ()");
  m.def("layer_norm_fwd(Tensor x, Tensor? gamma, Tensor? beta, Tensor? res, float eps) -> "
        "(Tensor, Tensor, Tensor)");
  m.def("layer_norm_bwd(Tensor dy, Tensor x, Tensor mean, Tensor rstd, Tensor? gamma) -> "
        "(Tensor, Tensor, Tensor)");
  m.def("bn_reduce(Tensor x, Tensor? dy, Tensor center, Tensor? rstd, Tensor? gamma, "
        "Tensor? beta, bool relu, int mode, float drop_p=0., int seed=0) -> Tensor");
  m.def("bn_apply(Tensor x, Tensor? dy, Tensor mean, Tensor rstd, Tensor? gamma, Tensor? beta, "
        "Tensor? c1, Tensor? c2, bool relu, int mode, float drop_p=0., int seed=0) -> Tensor");
  m.def("dual_gemm(Tensor A1, Tensor B1t, Tensor? A2, Tensor? B2t, Tensor? bias, Tensor? cin, "
        "Tensor(a!) out, Tensor(b!)? mask_out, Tensor? mask_in, bool relu) -> ()");
  m.def("tile32_mask_words(int M, int N) -> int", &tile32_mask_words_op);
  m.def("gather_add_act(Tensor? Y, Tensor? P, Tensor? src, Tensor? Q, Tensor? dst, Tensor? gin, "
        "Tensor(a!) out, int act) -> ()");
  m.def(
      "spmm(Tensor rowptr, Tensor col, Tensor? edge_weight, Tensor? col_scale, "
      "Tensor? row_scale, Tensor x, Tensor(a!) out, int heads, int head_dim, float beta, "
      "int cap=0, Tensor? row_map=None) -> ()");
  m.def("spmm_hub_partials(Tensor seg_beg, Tensor seg_end, Tensor col, Tensor? edge_weight, "
        "Tensor? col_scale, Tensor x, Tensor(a!) partials) -> ()");
  m.def("spmm_hub_reduce(Tensor partials, Tensor hub_seg_ptr, Tensor hub_rows, "
        "Tensor? row_scale, Tensor(a!) out) -> ()");
  m.def("copy_rows(Tensor x, Tensor? src_idx, Tensor? dst_idx, Tensor(a!) out, "
        "bool accumulate) -> ()");
  m.def("masked_gather_rows(Tensor x, Tensor idx, Tensor mask, int value, Tensor(a!) out) -> ()");
  m.def("edge_softmax_fwd(Tensor rowptr, Tensor scores, Tensor(a!) alpha) -> ()");
  m.def("edge_softmax_bwd(Tensor rowptr, Tensor alpha, Tensor grad, Tensor(a!) ds) -> ()");
}

TORCH_LIBRARY_IMPL(dgraph_amd, CUDA, m) {
  m.impl("spmm", &dgraph::spmm);
  m.impl("spmm_hub_partials", &dgraph::spmm_hub_partials_op);
  m.impl("spmm_hub_reduce", &dgraph::spmm_hub_reduce_op);
  m.impl("copy_rows", &dgraph::copy_rows_op);
  m.impl("masked_gather_rows", &dgraph::masked_gather_rows_op);
  m.impl("edge_softmax_fwd", &dgraph::edge_softmax_fwd_op);
  m.impl("edge_softmax_bwd", &dgraph::edge_softmax_bwd_op);
  m.impl("bias_relu_pack", &dgraph::bias_relu_pack_op);
  m.impl("relu_mask_bwd", &dgraph::relu_mask_bwd_op);
  m.impl("col_sum", &dgraph::col_sum_op);
  m.impl("bias_act", &dgraph::bias_act_op);
  m.impl("bias_act_bwd", &dgraph::bias_act_bwd_op);
  m.impl("row_scale_cols", &dgraph::row_scale_cols_op);
  m.impl("row_scale_colsum", &dgraph::row_scale_colsum_op);
  m.impl("pair_relu", &dgraph::pair_relu_op);
  m.impl("gather_add_act", &dgraph::gather_add_act_op);
  m.impl("layer_norm_fwd", &dgraph::layer_norm_fwd_op);
  m.impl("dual_gemm", &dgraph::dual_gemm_op);
  m.impl("layer_norm_bwd", &dgraph::layer_norm_bwd_op);
  m.impl("bn_reduce", &dgraph::bn_reduce_op);
  m.impl("bn_apply", &dgraph::bn_apply_op);
}
