// dgraph_amd — LDS-DMA helpers (gfx950 global_load_lds_dwordx4) shared by the MFMA kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dgraph {

typedef __attribute__((address_space(3))) void* lds_void_ptr;

// One LDS-DMA wave-instruction: each ACTIVE lane's 16 B from `src` land at lds_base + 16 l
// (lane-linear image; lds_base must be wave-uniform). Issued as inline asm on purpose:
// hipcc tracks __builtin_amdgcn_global_load_lds as an LDS write it cannot disambiguate and
// then waits vmcnt(0) before every ds_read in its scope; completion is the caller's counted
// wait (wait_vmcnt) + barrier instead.
__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_ptr)lds_base)));
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(src), "s"(l)
               : "memory", "m0");
}

// s_waitcnt vmcnt(n) (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14; expcnt/lgkmcnt left at
// their maxima, i.e. not waited for)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// End of a dynamically scheduled persistent block (work_counter, kernels.h): thread 0
// counts the block done after its last pull of ctr[0]; the grid's last block resets the
// pair, so the next launch on the stream (or the next replay of a captured graph) starts
// from zero. Call once per block, from every thread, after the block's last work pull.
__device__ __forceinline__ void work_counter_release(int* ctr) {
  if (ctr == nullptr || threadIdx.x != 0) return;
  __threadfence();  // this block's pulls of ctr[0] are ordered before its done count
  const int d = atomicAdd(ctr + 1, 1);
  if (d == static_cast<int>(gridDim.x) - 1) {
    __threadfence();
    atomicExch(ctr, 0);
    atomicExch(ctr + 1, 0);
  }
}

}  // namespace dgraph
