// dgraph_amd — host-side plan validation (pure C++17: no torch, no HIP).
//
// The hand-written kernels trust their index structures: a CSR column id out of range is
// an out-of-bounds gather, a duplicated output row in a row-compacted pass (row_map) is
// two waves writing the same row (a write race), an overlapping hub-split segment is a
// double count. These checks run on the host before such a plan is first launched
// (DGRAPH_CHECK_PLANS=1, utils/diagnostics.py) and are compiled a second time, with the
// host test driver, under AddressSanitizer + UBSan and ThreadSanitizer
// (csrc/host/Makefile `sanitize`, CMake option DGRAPH_HOST_SANITIZE): GPU sanitizers are
// not available on the target pool, so the native host code is what gets sanitized.
//
// Large inputs (papers100M: 3.2e9 column ids) are scanned by `threads` std::threads over
// disjoint ranges; every result is reduced after join (no shared mutable state).
#pragma once
#include <cstdint>
#include <string>

namespace dgraph {
namespace host {

struct CheckResult {
  bool ok = true;
  int64_t where = -1;  // first offending index (row, entry or segment)
  std::string what;
};

// rowptr[nrows+1] monotone, rowptr[0] == 0, rowptr[nrows] == nnz; every col in [0, ncols).
// col is int32 (col_bytes == 4) or int64 (8).
CheckResult check_csr(const int64_t* rowptr, int64_t nrows, const void* col, int col_bytes,
                      int64_t nnz, int64_t ncols, int threads = 0);

// row_map[n]: every entry in [0, nrows_out) and no entry twice (a duplicate would make two
// row groups of a compacted pass write the same output row).
CheckResult check_row_map(const int64_t* row_map, int64_t n, int64_t nrows_out,
                          int threads = 0);

// Hub split: segment s covers entries [seg_lo[s], seg_hi[s]) of CSR row seg_row[s]; the
// main pass keeps the first `head` entries of a hub row, so a row's segments must be
// sorted, contiguous, non-overlapping and together cover exactly
// [rowptr[r] + head, rowptr[r+1]); rows must be strictly increasing.
CheckResult check_hub_split(const int64_t* rowptr, int64_t nrows, const int64_t* seg_row,
                            const int64_t* seg_lo, const int64_t* seg_hi, int64_t nseg,
                            int64_t head = 0);

// All-to-all-v splits: sums equal the buffer sizes, no negative count.
CheckResult check_splits(const int64_t* send, const int64_t* recv, int world,
                         int64_t total_send, int64_t total_recv);

}  // namespace host
}  // namespace dgraph
