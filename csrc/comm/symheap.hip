// dgraph_amd — one-sided symmetric heap over HIP IPC (the NVSHMEM replacement, N3/N4).
//
// rocSHMEM is not installed, so every rank hipMalloc's a heap of the SAME size (the max
// over ranks: the reference's collective nvshmem_malloc had mismatched sizes, D4),
// exports an IPC handle (dmabuf under HSA_ENABLE_IPC_MODE_LEGACY=0), and maps every peer's
// heap into its address space. Kernels then read/write peer memory directly over xGMI:
//
//   heap_get_rows : out[i] = heap_of(owner[i])[base_off + row[i]*ld, +F)   (K15: remote get)
//   heap_put_rows : heap_of(peer)[dst_off + (remote_off[peer] + j)*ld] = src[send_off[peer] + j]
//                   for every peer segment (one-sided put at remote_offsets, HaloExchange)
//
// One wavefront moves G = 64/LPR rows per step with 16-B loads/stores; the peer table is a
// small device array of base pointers. Completion: the host drains the stream and joins a
// process-group barrier (writes from a peer are visible to a rank once the peer's kernel
// has completed and both have passed the barrier; stores to peer memory are made visible
// with a system-scope release at kernel end).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../common.h"
#include "comm.h"

namespace dgraph {
namespace {

// Both kernels keep U rows per lane group in flight (all index loads, then all row loads,
// then the stores): a remote row read over xGMI has several times the latency of a local
// one, and one row per iteration left each wave a single dependent index->load->store
// chain (the local copy_rows pack with that shape ran at ~2 TB/s, at 4 rows 5.9 TB/s).
template <typename T, int VEC, int LPR, int U>
__global__ __launch_bounds__(256) void heap_get_rows_kernel(
    const uint64_t* __restrict__ peer_base, int64_t base_off, const int64_t* __restrict__ owner,
    const int64_t* __restrict__ row, T* __restrict__ out, int64_t ld_src, int64_t ld_out,
    int64_t n, int F) {
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & 63;
  const int g = lane / LPR, l = lane % LPR;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t base = wave * G * U; base < n; base += nwaves * G * U) {
    const T* src[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * G + g;
      src[u] = i < n ? reinterpret_cast<const T*>(peer_base[owner[i]] + base_off) + row[i] * ld_src
                     : nullptr;
    }
    for (int f = l * VEC; f < F; f += LPR * VEC) {
      float v[U][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (src[u]) load_vec_f32<T, VEC>(src[u] + f, v[u]);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (src[u]) store_vec_f32<T, VEC>(out + (base + u * G + g) * ld_out + f, v[u]);
    }
  }
}

template <typename T, int VEC, int LPR, int U>
__global__ __launch_bounds__(256) void heap_put_rows_kernel(
    const uint64_t* __restrict__ peer_base, int64_t dst_off, const int64_t* __restrict__ row_peer,
    const int64_t* __restrict__ row_dst, const T* __restrict__ src, int64_t ld_src,
    int64_t ld_dst, int64_t n, int F) {
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & 63;
  const int g = lane / LPR, l = lane % LPR;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t base = wave * G * U; base < n; base += nwaves * G * U) {
    T* dst[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * G + g;
      dst[u] = i < n ? reinterpret_cast<T*>(peer_base[row_peer[i]] + dst_off) + row_dst[i] * ld_dst
                     : nullptr;
    }
    for (int f = l * VEC; f < F; f += LPR * VEC) {
      float v[U][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (dst[u]) load_vec_f32<T, VEC>(src + (base + u * G + g) * ld_src + f, v[u]);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (dst[u]) store_vec_f32<T, VEC>(dst[u] + f, v[u]);
    }
  }
  // make this block's peer stores visible system-wide before the kernel retires
  __threadfence_system();
}

// ---------------------------------------------------------------------------------------
// Stream-ordered completion (the nvshmemx_quiet_on_stream / barrier_all_on_stream /
// signal_wait_until counterpart). Each rank's heap starts with flag words
// flags[kind][W] (uint64). A producer, after its put/copy kernels on the same stream,
// runs heap_signal: lane p stores `epoch` into flags[kind][me] of peer p's heap with a
// system-scope RELEASE (the data stores of the earlier kernels on this stream were
// retired before this kernel started, and each put block ended with a system fence). A
// consumer runs heap_wait: lane q spins on its OWN heap's flags[kind][q] with a
// system-scope ACQUIRE until it reaches `epoch` (monotonic epochs: no reset races).
// All flag traffic is vector memory (global atomics), never scalar. The spin is bounded:
// after max_spins polls (with s_sleep) the lane gives up, sets *timed_out and exits, so
// the grid always drains (the host raises on the flag).
__global__ __launch_bounds__(64) void heap_signal_kernel(const uint64_t* __restrict__ peer_base,
                                                         int64_t flag_off, int me, int world,
                                                         uint64_t epoch, int self_too) {
  const int p = threadIdx.x;
  if (p >= world || (p == me && !self_too)) return;
  uint64_t* f = reinterpret_cast<uint64_t*>(peer_base[p] + flag_off) + me;
  __hip_atomic_store(f, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void heap_wait_kernel(const uint64_t* __restrict__ flags,
                                                       int me, int world, uint64_t epoch,
                                                       int64_t max_spins, int self_too,
                                                       int* __restrict__ timed_out) {
  const int q = threadIdx.x;
  if (q >= world || (q == me && !self_too)) return;
  int64_t spins = 0;
  while (__hip_atomic_load(flags + q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
    if (++spins >= max_spins) {
      // system scope: the word may be pinned host memory polled by the host
      __hip_atomic_store(timed_out, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

inline int pick_lpr(int lanes) {
  return lanes <= 4 ? 4 : lanes <= 8 ? 8 : lanes <= 16 ? 16 : lanes <= 32 ? 32 : 64;
}

template <typename T>
hipError_t launch_get(const uint64_t* pb, int64_t off, const int64_t* own, const int64_t* row,
                      void* out, int64_t lds, int64_t ldo, int64_t n, int F, hipStream_t st) {
  dim3 block(256), grid(static_cast<unsigned>(cap_blocks((n + 63) / 64, 256 * 16)));
  constexpr int V = 16 / sizeof(T);
  const bool vec = F % V == 0 && lds % V == 0 && ldo % V == 0;
  const int lpr = pick_lpr(vec ? F / V : F);
#define DG_GET(VV, L)                                                                        \
  hipLaunchKernelGGL((heap_get_rows_kernel<T, VV, L, 4>), grid, block, 0, st, pb, off, own, row, \
                     static_cast<T*>(out), lds, ldo, n, F)
#define DG_GET_ALL(VV)                                        \
  switch (lpr) {                                              \
    case 4: DG_GET(VV, 4); break;                             \
    case 8: DG_GET(VV, 8); break;                             \
    case 16: DG_GET(VV, 16); break;                           \
    case 32: DG_GET(VV, 32); break;                           \
    default: DG_GET(VV, 64); break;                           \
  }
  if (vec) { DG_GET_ALL(V) } else { DG_GET_ALL(1) }
#undef DG_GET_ALL
#undef DG_GET
  return hipGetLastError();
}

template <typename T>
hipError_t launch_put(const uint64_t* pb, int64_t off, const int64_t* rp, const int64_t* rd,
                      const void* src, int64_t lds, int64_t ldd, int64_t n, int F, hipStream_t st) {
  dim3 block(256), grid(static_cast<unsigned>(cap_blocks((n + 63) / 64, 256 * 16)));
  constexpr int V = 16 / sizeof(T);
  const bool vec = F % V == 0 && lds % V == 0 && ldd % V == 0;
  const int lpr = pick_lpr(vec ? F / V : F);
#define DG_PUT(VV, L)                                                                       \
  hipLaunchKernelGGL((heap_put_rows_kernel<T, VV, L, 4>), grid, block, 0, st, pb, off, rp, rd, \
                     static_cast<const T*>(src), lds, ldd, n, F)
#define DG_PUT_ALL(VV)                                        \
  switch (lpr) {                                              \
    case 4: DG_PUT(VV, 4); break;                             \
    case 8: DG_PUT(VV, 8); break;                             \
    case 16: DG_PUT(VV, 16); break;                           \
    case 32: DG_PUT(VV, 32); break;                           \
    default: DG_PUT(VV, 64); break;                           \
  }
  if (vec) { DG_PUT_ALL(V) } else { DG_PUT_ALL(1) }
#undef DG_PUT_ALL
#undef DG_PUT
  return hipGetLastError();
}

}  // namespace

hipError_t heap_signal(const uint64_t* peer_base, int64_t flag_off, int me, int world,
                       uint64_t epoch, bool self_too, hipStream_t st) {
  if (world <= 0 || world > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(heap_signal_kernel, dim3(1), dim3(64), 0, st, peer_base, flag_off, me,
                     world, epoch, self_too ? 1 : 0);
  return hipGetLastError();
}

hipError_t heap_wait(const uint64_t* flags, int me, int world, uint64_t epoch,
                     int64_t max_spins, bool self_too, int* timed_out, hipStream_t st) {
  if (world <= 0 || world > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(heap_wait_kernel, dim3(1), dim3(64), 0, st, flags, me, world, epoch,
                     max_spins, self_too ? 1 : 0, timed_out);
  return hipGetLastError();
}

hipError_t heap_get_rows(DType dt, const uint64_t* peer_base, int64_t base_off,
                         const int64_t* owner, const int64_t* row, void* out, int64_t ld_src,
                         int64_t ld_out, int64_t n, int F, hipStream_t st) {
  if (n <= 0 || F <= 0) return hipSuccess;
  if (dt == DType::F32)
    return launch_get<float>(peer_base, base_off, owner, row, out, ld_src, ld_out, n, F, st);
  return launch_get<uint16_t>(peer_base, base_off, owner, row, out, ld_src, ld_out, n, F, st);
}

hipError_t heap_put_rows(DType dt, const uint64_t* peer_base, int64_t dst_off,
                         const int64_t* row_peer, const int64_t* row_dst, const void* src,
                         int64_t ld_src, int64_t ld_dst, int64_t n, int F, hipStream_t st) {
  if (n <= 0 || F <= 0) return hipSuccess;
  if (dt == DType::F32)
    return launch_put<float>(peer_base, dst_off, row_peer, row_dst, src, ld_src, ld_dst, n, F, st);
  return launch_put<uint16_t>(peer_base, dst_off, row_peer, row_dst, src, ld_src, ld_dst, n, F,
                              st);
}

// ---------------------------------------------------------------------------------------
// Link-time model of a loopback exchange (single-process rehearsal of a W-way rank): one
// lane of each one-wave block waits `ticks` of the constant-rate wall clock (s_memrealtime,
// read by wall_clock64) with s_sleep between polls, so the stream it runs on is held for
// the time the exchange's largest per-peer message would take on one xGMI link. Each block
// holds a wave slot of a CU (and no memory bandwidth) — several blocks stand for the CUs a
// collective's kernel occupies while it moves data.
__global__ __launch_bounds__(64) void link_delay_kernel(uint64_t ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}

namespace {
uint64_t us_to_ticks(double us) {
  static int khz = 0;
  if (khz == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        khz <= 0)
      khz = 100000;  // 100 MHz
  }
  const double t = us * 1e-3 * static_cast<double>(khz);
  return t > 1.8e19 ? ~0ull : static_cast<uint64_t>(t);
}

// The modelled collective as ONE kernel: `blocks` workgroups copy the message (16-B
// vectors, grid-stride; a byte tail) — the HBM traffic a real transfer puts on both ends —
// and the first `hold` of them (RCCL moves an all-to-all with one workgroup per channel)
// then stay resident until `ticks` have passed since they started, so the transfer takes
// max(copy, link time) and the data moves while the link time runs, as on a real link.
__global__ __launch_bounds__(256) void link_copy_kernel(const uint8_t* __restrict__ src,
                                                        uint8_t* __restrict__ dst,
                                                        int64_t nbytes, uint64_t ticks,
                                                        int hold) {
  const uint64_t t0 = wall_clock64();
  const int64_t nv = nbytes >> 4;
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t step = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  int64_t i = tid;
  for (; i + 3 * step < nv; i += 4 * step) {  // four 16-B loads in flight per lane
    const uint4 a = s4[i], b = s4[i + step], c = s4[i + 2 * step], d = s4[i + 3 * step];
    d4[i] = a;
    d4[i + step] = b;
    d4[i + 2 * step] = c;
    d4[i + 3 * step] = d;
  }
  for (; i < nv; i += step) d4[i] = s4[i];
  for (int64_t j = (nv << 4) + tid; j < nbytes; j += step) dst[j] = src[j];
  if (threadIdx.x != 0 || static_cast<int>(blockIdx.x) >= hold) return;
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}
}  // namespace

hipError_t link_delay(double us, hipStream_t st, int blocks) {
  if (!(us > 0.0)) return hipSuccess;
  const uint64_t ticks = us_to_ticks(us);
  hipLaunchKernelGGL(link_delay_kernel, dim3(blocks > 0 ? blocks : 1), dim3(64), 0, st, ticks);
  return hipGetLastError();
}

hipError_t link_copy(const void* src, void* dst, int64_t nbytes, double us, hipStream_t st,
                     int blocks, int hold) {
  if (nbytes < 0) return hipErrorInvalidValue;
  const bool aligned = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) &
                        15) == 0;
  if (!aligned) return hipErrorInvalidValue;
  const uint64_t ticks = us > 0.0 ? us_to_ticks(us) : 0;
  hipLaunchKernelGGL(link_copy_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st,
                     static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), nbytes,
                     ticks, hold);
  return hipGetLastError();
}

}  // namespace dgraph
