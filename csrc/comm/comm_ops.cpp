// dgraph_amd — native communication ops: IPC symmetric heap and the RCCL plan executor.
//
// Symmetric heap (replaces the NVSHMEM runtime of DGraph/distributed/nvshmem/, N3/N4):
//   heap_alloc / ipc_get_handle / ipc_open_handle / ipc_close manage one hipMalloc'd region
//   per rank mapped into every peer; heap_get_rows / heap_put_rows are the one-sided
//   remote get / put kernels (symheap.hip).
//
// RCCL plan executor (the two-sided transport under a CompiledPlan, N7): a dedicated RCCL
// communicator driven directly with grouped ncclSend/ncclRecv. Compared with
// ProcessGroupNCCL::alltoall_base it skips zero-size peers, takes host-cached row splits
// (no device->host split copies), moves several tensors in one group call, and launches on
// the caller's current stream (so it composes with HIP-stream overlap and graph capture).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <rccl/rccl.h>
#include <torch/library.h>

#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../check.h"
#include "comm.h"

#define DG_NCCL_CHECK(expr)                                                               \
  do {                                                                                    \
    ncclResult_t _r = (expr);                                                             \
    TORCH_CHECK(_r == ncclSuccess, "dgraph_amd RCCL error: ", ncclGetErrorString(_r),     \
                " at " #expr);                                                            \
  } while (0)

namespace dgraph {
namespace {

hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

DType dtype_of(const at::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return DType::F32;
  if (t.scalar_type() == at::kBFloat16) return DType::BF16;
  TORCH_CHECK(false, "dgraph_amd: unsupported dtype ", t.scalar_type());
}

// ------------------------------------------------------------------ symmetric heap
// fine = true: fine-grained device memory (hipDeviceMallocFinegrained): peers' writes over
// xGMI are coherent for this GPU's readers at any time, not only at kernel boundaries
// after a system-scope acquire — the heap's alternative when coarse-grained IPC memory
// turns out not to be (the one-sided probe of bench.py measures both)
at::Tensor heap_alloc(int64_t nbytes, int64_t device, bool fine) {
  TORCH_CHECK(nbytes > 0, "heap_alloc: nbytes must be positive");
  c10::DeviceGuard g(c10::Device(c10::kCUDA, static_cast<c10::DeviceIndex>(device)));
  void* p = nullptr;
  if (fine)
    DG_HIP_CHECK(hipExtMallocWithFlags(&p, static_cast<size_t>(nbytes),
                                       hipDeviceMallocFinegrained));
  else
    DG_HIP_CHECK(hipMalloc(&p, static_cast<size_t>(nbytes)));
  DG_HIP_CHECK(hipMemset(p, 0, static_cast<size_t>(nbytes)));
  auto opts = at::TensorOptions().dtype(at::kByte).device(c10::kCUDA, device);
  return at::from_blob(
      p, {nbytes}, [](void* q) { (void)hipFree(q); }, opts);
}

at::Tensor ipc_get_handle(const at::Tensor& heap) {
  TORCH_CHECK(heap.is_cuda(), "ipc_get_handle: heap must be a GPU tensor");
  c10::DeviceGuard g(heap.device());
  hipIpcMemHandle_t h;
  DG_HIP_CHECK(hipIpcGetMemHandle(&h, heap.data_ptr()));
  auto out = at::empty({static_cast<int64_t>(sizeof(h))}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), &h, sizeof(h));
  return out;
}

int64_t ipc_open_handle(const at::Tensor& handle, int64_t device) {
  TORCH_CHECK(!handle.is_cuda() && handle.numel() == sizeof(hipIpcMemHandle_t),
              "ipc_open_handle: expected a host uint8 tensor of ", sizeof(hipIpcMemHandle_t),
              " bytes");
  c10::DeviceGuard g(c10::Device(c10::kCUDA, static_cast<c10::DeviceIndex>(device)));
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.contiguous().data_ptr(), sizeof(h));
  void* p = nullptr;
  DG_HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  return static_cast<int64_t>(reinterpret_cast<uintptr_t>(p));
}

void ipc_close(int64_t ptr) {
  if (ptr) DG_HIP_CHECK(hipIpcCloseMemHandle(reinterpret_cast<void*>(static_cast<uintptr_t>(ptr))));
}

int64_t tensor_ptr(const at::Tensor& t) {
  return static_cast<int64_t>(reinterpret_cast<uintptr_t>(t.data_ptr()));
}

void check_table(const at::Tensor& table, const at::Tensor& ref) {
  TORCH_CHECK(table.is_cuda() && table.device() == ref.device() &&
                  table.scalar_type() == at::kLong && table.is_contiguous(),
              "peer table must be a contiguous int64 tensor on the data's device");
}

void check_idx(const at::Tensor& idx, const at::Tensor& ref, int64_t n, const char* name) {
  TORCH_CHECK(idx.is_cuda() && idx.device() == ref.device() && idx.scalar_type() == at::kLong &&
                  idx.is_contiguous() && idx.numel() == n,
              name, " must be a contiguous int64 GPU tensor with ", n, " entries");
}

// out[i] = peer(owner[i]).heap[base_off + row[i] * ld_src * esize, +F)
void heap_get_rows_op(const at::Tensor& table, int64_t base_off, const at::Tensor& owner,
                      const at::Tensor& row, const at::Tensor& out, int64_t ld_src) {
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1, "out must be [n, F] with unit stride");
  const int64_t n = out.size(0);
  check_table(table, out);
  check_idx(owner, out, n, "owner");
  check_idx(row, out, n, "row");
  c10::DeviceGuard g(out.device());
  DG_HIP_CHECK(heap_get_rows(dtype_of(out), reinterpret_cast<const uint64_t*>(table.data_ptr()),
                             base_off, owner.data_ptr<int64_t>(), row.data_ptr<int64_t>(),
                             out.data_ptr(), ld_src, out.stride(0), n,
                             static_cast<int>(out.size(1)), cur_stream(out)));
}

void heap_put_rows_op(const at::Tensor& table, int64_t dst_off, const at::Tensor& row_peer,
                      const at::Tensor& row_dst, const at::Tensor& src, int64_t ld_dst) {
  TORCH_CHECK(src.dim() == 2 && src.stride(1) == 1, "src must be [n, F] with unit stride");
  const int64_t n = src.size(0);
  check_table(table, src);
  check_idx(row_peer, src, n, "row_peer");
  check_idx(row_dst, src, n, "row_dst");
  c10::DeviceGuard g(src.device());
  DG_HIP_CHECK(heap_put_rows(dtype_of(src), reinterpret_cast<const uint64_t*>(table.data_ptr()),
                             dst_off, row_peer.data_ptr<int64_t>(), row_dst.data_ptr<int64_t>(),
                             src.data_ptr(), src.stride(0), ld_dst, n,
                             static_cast<int>(src.size(1)), cur_stream(src)));
}

void heap_signal_op(const at::Tensor& table, int64_t flag_off, int64_t me, int64_t world,
                    int64_t epoch, bool self_too) {
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kLong && table.numel() == world,
              "table must be the int64 GPU peer table of the group");
  c10::DeviceGuard g(table.device());
  DG_HIP_CHECK(heap_signal(reinterpret_cast<const uint64_t*>(table.data_ptr()), flag_off,
                           static_cast<int>(me), static_cast<int>(world),
                           static_cast<uint64_t>(epoch), self_too, cur_stream(table)));
}

void heap_wait_op(const at::Tensor& flags, int64_t me, int64_t world, int64_t epoch,
                  int64_t max_spins, bool self_too, const at::Tensor& timed_out) {
  TORCH_CHECK(flags.is_cuda() && flags.scalar_type() == at::kLong && flags.numel() >= world &&
                  flags.is_contiguous(),
              "flags must be a contiguous int64 GPU tensor of >= world words");
  TORCH_CHECK(timed_out.scalar_type() == at::kInt && (timed_out.is_cuda() || timed_out.is_pinned()),
              "timed_out must be an int32 GPU tensor or pinned host tensor");
  c10::DeviceGuard g(flags.device());
  int* flag = timed_out.data_ptr<int>();
  if (!timed_out.is_cuda()) {
    // pinned host word: the wait kernel reports a timeout straight into host memory, so
    // the host can poll it on every call without a device sync
    void* dptr = nullptr;
    DG_HIP_CHECK(hipHostGetDevicePointer(&dptr, flag, 0));
    flag = static_cast<int*>(dptr);
  }
  DG_HIP_CHECK(heap_wait(reinterpret_cast<const uint64_t*>(flags.data_ptr()),
                         static_cast<int>(me), static_cast<int>(world),
                         static_cast<uint64_t>(epoch), max_spins, self_too, flag,
                         cur_stream(flags)));
}

// ------------------------------------------------------------------ RCCL executor
struct CommEntry {
  ncclComm_t comm;
  int rank, world;
};
std::mutex g_mu;
std::unordered_map<int64_t, CommEntry> g_comms;
int64_t g_next = 1;

CommEntry get_comm(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_comms.find(h);
  TORCH_CHECK(it != g_comms.end(), "dgraph_amd: unknown RCCL communicator handle ", h);
  return it->second;
}

at::Tensor rccl_unique_id() {
  ncclUniqueId id;
  DG_NCCL_CHECK(ncclGetUniqueId(&id));
  auto out = at::empty({NCCL_UNIQUE_ID_BYTES}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), &id, NCCL_UNIQUE_ID_BYTES);
  return out;
}

int64_t rccl_comm_init(const at::Tensor& uid, int64_t world, int64_t rank, int64_t device) {
  TORCH_CHECK(uid.numel() == NCCL_UNIQUE_ID_BYTES && !uid.is_cuda(), "bad RCCL unique id");
  c10::DeviceGuard g(c10::Device(c10::kCUDA, static_cast<c10::DeviceIndex>(device)));
  ncclUniqueId id;
  std::memcpy(&id, uid.contiguous().data_ptr(), NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm;
  DG_NCCL_CHECK(ncclCommInitRank(&comm, static_cast<int>(world), id, static_cast<int>(rank)));
  std::lock_guard<std::mutex> lk(g_mu);
  const int64_t h = g_next++;
  g_comms[h] = CommEntry{comm, static_cast<int>(rank), static_cast<int>(world)};
  return h;
}

void rccl_comm_destroy(int64_t h) {
  ncclComm_t comm;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_comms.find(h);
    if (it == g_comms.end()) return;
    comm = it->second.comm;
    g_comms.erase(it);
  }
  DG_NCCL_CHECK(ncclCommDestroy(comm));
}

ncclDataType_t nccl_type(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kByte: return ncclUint8;
    default: TORCH_CHECK(false, "dgraph_amd RCCL: unsupported dtype ", t.scalar_type());
  }
}

// Variable all-to-all of several row-major tensors in ONE grouped call.
//   sends[k] : [sum(send_rows), F_k]   recvs[k] : [sum(recv_rows), F_k]
//   send_rows / recv_rows : host int64 [world] row counts (the plan's cached splits)
void rccl_alltoallv(int64_t h, at::TensorList sends, at::TensorList recvs,
                    const at::Tensor& send_rows, const at::Tensor& recv_rows) {
  const CommEntry c = get_comm(h);
  TORCH_CHECK(sends.size() == recvs.size() && !sends.empty(), "sends/recvs mismatch");
  TORCH_CHECK(!send_rows.is_cuda() && !recv_rows.is_cuda() && send_rows.numel() == c.world &&
                  recv_rows.numel() == c.world,
              "row splits must be host int64 tensors of length world");
  auto sr = send_rows.contiguous().to(at::kLong);
  auto rr = recv_rows.contiguous().to(at::kLong);
  const int64_t* s = sr.data_ptr<int64_t>();
  const int64_t* r = rr.data_ptr<int64_t>();
  const at::Tensor& ref = sends[0];
  c10::DeviceGuard g(ref.device());
  hipStream_t st = cur_stream(ref);
  DG_NCCL_CHECK(ncclGroupStart());
  for (size_t k = 0; k < sends.size(); ++k) {
    const at::Tensor& x = sends[k];
    const at::Tensor& y = recvs[k];
    TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.scalar_type() == y.scalar_type(),
                "alltoallv tensors must be contiguous and of one dtype");
    // elements per row (tensors may be 1-D: width 1)
    const int64_t wx = x.dim() > 1 ? x.numel() / std::max<int64_t>(1, x.size(0)) : 1;
    const int64_t wy = y.dim() > 1 ? y.numel() / std::max<int64_t>(1, y.size(0)) : 1;
    TORCH_CHECK(wx == wy || x.numel() == 0 || y.numel() == 0, "row width mismatch");
    const int64_t width = x.numel() ? wx : wy;
    const auto dt = nccl_type(x);
    const size_t es = x.element_size();
    const char* xp = static_cast<const char*>(x.data_ptr());
    char* yp = static_cast<char*>(y.data_ptr());
    int64_t so = 0, ro = 0;
    for (int p = 0; p < c.world; ++p) {
      if (s[p] > 0)
        DG_NCCL_CHECK(ncclSend(xp + so * width * es, static_cast<size_t>(s[p] * width), dt, p,
                               c.comm, st));
      if (r[p] > 0)
        DG_NCCL_CHECK(ncclRecv(yp + ro * width * es, static_cast<size_t>(r[p] * width), dt, p,
                               c.comm, st));
      so += s[p];
      ro += r[p];
    }
    TORCH_CHECK(so * width <= x.numel() && ro * width <= y.numel(), "splits exceed tensors");
  }
  DG_NCCL_CHECK(ncclGroupEnd());
}

void rccl_allreduce(int64_t h, const at::Tensor& t) {
  const CommEntry c = get_comm(h);
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "allreduce tensor must be contiguous GPU");
  c10::DeviceGuard g(t.device());
  DG_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_type(t), ncclSum,
                              c.comm, cur_stream(t)));
}

// Hold the current stream of `device` for `us` microseconds (device-side wait; the link
// model of the single-process rehearsal's loopback exchange, comm/alltoallv.py)
void link_delay_op(double us, int64_t device, int64_t blocks) {
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, static_cast<c10::DeviceIndex>(device)));
  DG_HIP_CHECK(link_delay(us, c10::hip::getCurrentHIPStream(device).stream(),
                          static_cast<int>(blocks)));
}

// The rehearsal's modelled transfer: dst <- src (same byte count, contiguous) by `blocks`
// workgroups that stay resident for at least `us` (comm/alltoallv.py)
void link_copy_op(const at::Tensor& src, at::Tensor& dst, double us, int64_t blocks,
                  int64_t hold) {
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.device() == dst.device(),
              "link_copy: tensors on one GPU");
  TORCH_CHECK(src.is_contiguous() && dst.is_contiguous(), "link_copy: contiguous tensors");
  const int64_t nb = src.numel() * src.element_size();
  TORCH_CHECK(nb == dst.numel() * dst.element_size(), "link_copy: byte counts differ");
  c10::DeviceGuard g(src.device());
  DG_HIP_CHECK(link_copy(src.data_ptr(), dst.data_ptr(), nb, us,
                         c10::hip::getCurrentHIPStream(src.device().index()).stream(),
                         static_cast<int>(blocks), static_cast<int>(hold)));
}

}  // namespace
}  // namespace dgraph

TORCH_LIBRARY_FRAGMENT(dgraph_amd, m) {
  m.def("link_delay(float us, int device, int blocks=1) -> ()", &dgraph::link_delay_op);
  m.def("link_copy(Tensor src, Tensor(a!) dst, float us, int blocks, int hold) -> ()",
        &dgraph::link_copy_op);
  m.def("heap_alloc(int nbytes, int device, bool fine=False) -> Tensor", &dgraph::heap_alloc);
  m.def("ipc_get_handle(Tensor heap) -> Tensor", &dgraph::ipc_get_handle);
  m.def("ipc_open_handle(Tensor handle, int device) -> int", &dgraph::ipc_open_handle);
  m.def("ipc_close(int ptr) -> ()", &dgraph::ipc_close);
  m.def("tensor_ptr(Tensor t) -> int", &dgraph::tensor_ptr);
  m.def("heap_get_rows(Tensor table, int base_off, Tensor owner, Tensor row, Tensor(a!) out, "
        "int ld_src) -> ()",
        &dgraph::heap_get_rows_op);
  m.def("heap_put_rows(Tensor table, int dst_off, Tensor row_peer, Tensor row_dst, Tensor src, "
        "int ld_dst) -> ()",
        &dgraph::heap_put_rows_op);
  m.def("heap_signal(Tensor table, int flag_off, int me, int world, int epoch, "
        "bool self_too) -> ()",
        &dgraph::heap_signal_op);
  m.def("heap_wait(Tensor flags, int me, int world, int epoch, int max_spins, bool self_too, "
        "Tensor(a!) timed_out) -> ()",
        &dgraph::heap_wait_op);
  m.def("rccl_unique_id() -> Tensor", &dgraph::rccl_unique_id);
  m.def("rccl_comm_init(Tensor uid, int world, int rank, int device) -> int",
        &dgraph::rccl_comm_init);
  m.def("rccl_comm_destroy(int handle) -> ()", &dgraph::rccl_comm_destroy);
  m.def("rccl_alltoallv(int handle, Tensor[] sends, Tensor(a!)[] recvs, Tensor send_rows, "
        "Tensor recv_rows) -> ()",
        &dgraph::rccl_alltoallv);
  m.def("rccl_allreduce(int handle, Tensor(a!) t) -> ()", &dgraph::rccl_allreduce);
}
