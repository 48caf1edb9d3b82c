// dgraph_amd — native communication runtime (symmetric heap kernels, RCCL plan executor).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../kernels/kernels.h"

namespace dgraph {

// out[i, :F] = *(T*)(peer_base[owner[i]] + base_off)[row[i] * ld_src, +F)
hipError_t heap_get_rows(DType dt, const uint64_t* peer_base, int64_t base_off,
                         const int64_t* owner, const int64_t* row, void* out, int64_t ld_src,
                         int64_t ld_out, int64_t n, int F, hipStream_t st);

// *(T*)(peer_base[row_peer[i]] + dst_off)[row_dst[i] * ld_dst, +F) = src[i, :F]
hipError_t heap_put_rows(DType dt, const uint64_t* peer_base, int64_t dst_off,
                         const int64_t* row_peer, const int64_t* row_dst, const void* src,
                         int64_t ld_src, int64_t ld_dst, int64_t n, int F, hipStream_t st);

// stream-ordered completion flags (see symheap.hip): signal stores `epoch` into
// flags[me] of every peer's heap at flag_off (system-scope release); wait spins on the
// local flags[q] for every peer q until >= epoch (bounded; *timed_out = 1 on give-up)
hipError_t heap_signal(const uint64_t* peer_base, int64_t flag_off, int me, int world,
                       uint64_t epoch, bool self_too, hipStream_t st);
hipError_t heap_wait(const uint64_t* flags, int me, int world, uint64_t epoch,
                     int64_t max_spins, bool self_too, int* timed_out, hipStream_t st);

// hold stream `st` for `us` microseconds of device wall-clock time (rehearsal link model)
hipError_t link_delay(double us, hipStream_t st, int blocks = 1);
// copy nbytes src -> dst (16-B aligned) with `blocks` workgroups, `hold` of which stay
// resident until `us` have passed
hipError_t link_copy(const void* src, void* dst, int64_t nbytes, double us, hipStream_t st,
                     int blocks, int hold);

}  // namespace dgraph
