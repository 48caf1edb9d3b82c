// dgraph_amd — host-side plan validation (see plan_check.h).
#include "plan_check.h"

#include <algorithm>
#include <thread>
#include <vector>

namespace dgraph {
namespace host {
namespace {

int pick_threads(int threads, int64_t n) {
  if (threads <= 0) {
    const unsigned hc = std::thread::hardware_concurrency();
    threads = static_cast<int>(std::min<unsigned>(hc ? hc : 1, 16));
  }
  const int64_t per = int64_t(1) << 22;  // >= 4M items per thread
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(threads, (n + per - 1) / per)));
}

// Run body(lo, hi, &first_bad) over `threads` disjoint ranges of [0, n); return the
// smallest offending index any range reported (-1 if none).
template <typename Body>
int64_t parallel_first(int64_t n, int threads, Body body) {
  const int t = pick_threads(threads, n);
  std::vector<int64_t> bad(t, -1);
  std::vector<std::thread> pool;
  const int64_t chunk = (n + t - 1) / t;
  for (int i = 0; i < t; ++i) {
    const int64_t lo = std::min(n, i * chunk), hi = std::min(n, lo + chunk);
    if (t == 1) {
      body(lo, hi, &bad[i]);
    } else {
      pool.emplace_back([=, &bad] { body(lo, hi, &bad[i]); });
    }
  }
  for (auto& th : pool) th.join();
  int64_t first = -1;
  for (int64_t b : bad)
    if (b >= 0 && (first < 0 || b < first)) first = b;
  return first;
}

CheckResult fail(int64_t where, std::string what) {
  CheckResult r;
  r.ok = false;
  r.where = where;
  r.what = std::move(what);
  return r;
}

template <typename C>
int64_t first_bad_col(const C* col, int64_t nnz, int64_t ncols, int threads) {
  return parallel_first(nnz, threads, [=](int64_t lo, int64_t hi, int64_t* out) {
    for (int64_t i = lo; i < hi; ++i) {
      const int64_t c = static_cast<int64_t>(col[i]);
      if (c < 0 || c >= ncols) {
        *out = i;
        return;
      }
    }
  });
}

}  // namespace

CheckResult check_csr(const int64_t* rowptr, int64_t nrows, const void* col, int col_bytes,
                      int64_t nnz, int64_t ncols, int threads) {
  if (nrows < 0 || nnz < 0 || ncols < 0) return fail(-1, "negative size");
  if (rowptr == nullptr) return fail(-1, "rowptr is null");
  if (rowptr[0] != 0) return fail(0, "rowptr[0] != 0");
  if (rowptr[nrows] != nnz) return fail(nrows, "rowptr[nrows] != nnz");
  const int64_t bad_row = parallel_first(nrows, threads, [=](int64_t lo, int64_t hi, int64_t* out) {
    for (int64_t r = lo; r < hi; ++r) {
      if (rowptr[r + 1] < rowptr[r]) {
        *out = r;
        return;
      }
    }
  });
  if (bad_row >= 0) return fail(bad_row, "rowptr decreases");
  if (nnz == 0) return CheckResult{};
  if (col == nullptr) return fail(-1, "col is null");
  int64_t bad;
  if (col_bytes == 4) {
    bad = first_bad_col(static_cast<const int32_t*>(col), nnz, ncols, threads);
  } else if (col_bytes == 8) {
    bad = first_bad_col(static_cast<const int64_t*>(col), nnz, ncols, threads);
  } else {
    return fail(-1, "column ids must be int32 or int64");
  }
  if (bad >= 0) return fail(bad, "column id out of range");
  return CheckResult{};
}

CheckResult check_row_map(const int64_t* row_map, int64_t n, int64_t nrows_out, int threads) {
  if (n == 0) return CheckResult{};
  if (row_map == nullptr || nrows_out < 0) return fail(-1, "bad row map");
  const int64_t oob = parallel_first(n, threads, [=](int64_t lo, int64_t hi, int64_t* out) {
    for (int64_t i = lo; i < hi; ++i) {
      if (row_map[i] < 0 || row_map[i] >= nrows_out) {
        *out = i;
        return;
      }
    }
  });
  if (oob >= 0) return fail(oob, "row_map entry out of range");
  // uniqueness: one byte per output row (sequential: the first duplicate is reported)
  std::vector<uint8_t> seen(static_cast<size_t>(nrows_out), 0);
  for (int64_t i = 0; i < n; ++i) {
    uint8_t& s = seen[static_cast<size_t>(row_map[i])];
    if (s) return fail(i, "row_map maps two compacted rows to one output row (write race)");
    s = 1;
  }
  return CheckResult{};
}

CheckResult check_hub_split(const int64_t* rowptr, int64_t nrows, const int64_t* seg_row,
                            const int64_t* seg_lo, const int64_t* seg_hi, int64_t nseg,
                            int64_t head) {
  if (head < 0) return fail(-1, "negative head");
  int64_t s = 0;
  int64_t prev_row = -1;
  while (s < nseg) {
    const int64_t r = seg_row[s];
    if (r < 0 || r >= nrows) return fail(s, "segment row out of range");
    if (r <= prev_row) return fail(s, "hub rows not strictly increasing");
    if (rowptr[r + 1] - rowptr[r] <= head) return fail(s, "split row is not longer than head");
    int64_t pos = rowptr[r] + head;
    while (s < nseg && seg_row[s] == r) {
      if (seg_lo[s] != pos) return fail(s, "segment gap or overlap");
      if (seg_hi[s] <= seg_lo[s]) return fail(s, "empty or reversed segment");
      if (seg_hi[s] > rowptr[r + 1]) return fail(s, "segment runs past its row");
      pos = seg_hi[s];
      ++s;
    }
    if (pos != rowptr[r + 1]) return fail(s - 1, "segments do not cover the row");
    prev_row = r;
  }
  return CheckResult{};
}

CheckResult check_splits(const int64_t* send, const int64_t* recv, int world,
                         int64_t total_send, int64_t total_recv) {
  int64_t ss = 0, rs = 0;
  for (int p = 0; p < world; ++p) {
    if (send[p] < 0) return fail(p, "negative send count");
    if (recv[p] < 0) return fail(p, "negative recv count");
    ss += send[p];
    rs += recv[p];
  }
  if (ss != total_send) return fail(-1, "send splits do not sum to the send buffer");
  if (rs != total_recv) return fail(-1, "recv splits do not sum to the recv buffer");
  return CheckResult{};
}

}  // namespace host
}  // namespace dgraph
