// Host test driver for plan_check (built plain, under ASan+UBSan and under TSan by
// csrc/host/Makefile; run by tests/test_host_sanitize.py). Exit status 0 = all passed.
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#include "plan_check.h"

using dgraph::host::CheckResult;
namespace h = dgraph::host;

static int g_fail = 0;
#define EXPECT(cond, msg)                                        \
  do {                                                           \
    if (!(cond)) {                                               \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, msg); \
      ++g_fail;                                                  \
    }                                                            \
  } while (0)

int main() {
  std::mt19937_64 rng(7);
  // --- CSR: a random graph large enough to take the multi-threaded path ---
  const int64_t nrows = 1 << 20, ncols = 1 << 20;
  std::vector<int64_t> rowptr(nrows + 1, 0);
  for (int64_t r = 0; r < nrows; ++r) rowptr[r + 1] = rowptr[r] + static_cast<int64_t>(rng() % 17);
  const int64_t nnz = rowptr[nrows];
  std::vector<int32_t> col32(nnz);
  std::vector<int64_t> col64(nnz);
  for (int64_t i = 0; i < nnz; ++i) col64[i] = col32[i] = static_cast<int32_t>(rng() % ncols);
  for (int threads : {1, 4, 16}) {
    EXPECT(h::check_csr(rowptr.data(), nrows, col32.data(), 4, nnz, ncols, threads).ok, "valid int32");
    EXPECT(h::check_csr(rowptr.data(), nrows, col64.data(), 8, nnz, ncols, threads).ok, "valid int64");
  }
  col32[nnz - 1] = static_cast<int32_t>(ncols);
  CheckResult r = h::check_csr(rowptr.data(), nrows, col32.data(), 4, nnz, ncols, 8);
  EXPECT(!r.ok && r.where == nnz - 1, "last column out of range");
  col32[nnz - 1] = 0;
  col32[12345] = -1;
  r = h::check_csr(rowptr.data(), nrows, col32.data(), 4, nnz, ncols, 8);
  EXPECT(!r.ok && r.where == 12345, "negative column, first offender reported");
  col32[12345] = 0;
  std::swap(rowptr[500], rowptr[501]);
  if (rowptr[500] != rowptr[501]) {
    r = h::check_csr(rowptr.data(), nrows, col32.data(), 4, nnz, ncols, 8);
    EXPECT(!r.ok, "non-monotone rowptr");
  }
  std::swap(rowptr[500], rowptr[501]);
  EXPECT(!h::check_csr(rowptr.data(), nrows, col32.data(), 2, nnz, ncols).ok, "bad col width");
  std::vector<int64_t> empty_rp(5, 0);
  EXPECT(h::check_csr(empty_rp.data(), 4, nullptr, 4, 0, 0).ok, "empty CSR");

  // --- row maps ---
  std::vector<int64_t> rm(1 << 21);
  std::iota(rm.begin(), rm.end(), 0);
  std::shuffle(rm.begin(), rm.end(), rng);
  EXPECT(h::check_row_map(rm.data(), rm.size(), rm.size(), 8).ok, "permutation row map");
  rm[77] = rm[78];
  r = h::check_row_map(rm.data(), rm.size(), rm.size(), 8);
  EXPECT(!r.ok && (r.where == 78 || r.where == 77), "duplicate row = write race");
  rm[77] = static_cast<int64_t>(rm.size());
  EXPECT(!h::check_row_map(rm.data(), rm.size(), rm.size(), 8).ok, "row map out of range");

  // --- hub split: rows 3 and 9 split into segments ---
  std::vector<int64_t> rp = {0, 2, 4, 6, 106, 108, 110, 112, 114, 116, 316, 318};
  std::vector<int64_t> sr = {3, 3, 3, 9, 9}, lo = {6, 40, 80, 116, 216}, hi = {40, 80, 106, 216, 316};
  EXPECT(h::check_hub_split(rp.data(), 11, sr.data(), lo.data(), hi.data(), 5).ok, "valid split");
  lo[1] = 39;
  EXPECT(!h::check_hub_split(rp.data(), 11, sr.data(), lo.data(), hi.data(), 5).ok, "overlap");
  lo[1] = 40;
  hi[2] = 105;
  EXPECT(!h::check_hub_split(rp.data(), 11, sr.data(), lo.data(), hi.data(), 5).ok, "uncovered tail");
  hi[2] = 106;
  sr[3] = sr[4] = 2;
  EXPECT(!h::check_hub_split(rp.data(), 11, sr.data(), lo.data(), hi.data(), 5).ok, "rows unsorted");
  sr[3] = sr[4] = 9;
  // head = 34: the main pass keeps rowptr[r] .. +34, segments start after it
  std::vector<int64_t> lo2 = {40, 80, 150, 250}, hi2 = {80, 106, 250, 316}, sr2 = {3, 3, 9, 9};
  EXPECT(h::check_hub_split(rp.data(), 11, sr2.data(), lo2.data(), hi2.data(), 4, 34).ok, "head");
  EXPECT(!h::check_hub_split(rp.data(), 11, sr2.data(), lo2.data(), hi2.data(), 4, 33).ok,
         "head mismatch");

  // --- splits ---
  std::vector<int64_t> s = {3, 0, 5}, v = {1, 1, 1};
  EXPECT(h::check_splits(s.data(), v.data(), 3, 8, 3).ok, "valid splits");
  EXPECT(!h::check_splits(s.data(), v.data(), 3, 9, 3).ok, "send sum mismatch");
  s[1] = -1;
  EXPECT(!h::check_splits(s.data(), v.data(), 3, 7, 3).ok, "negative count");

  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("plan_check host tests passed\n");
  return 0;
}
