// Native RCCL communicator ("a C++ RCCL communicator (ncclCommInitRank, ncclAllReduce,
// ncclBroadcast) over one flat gradient buffer"; 5.8).  The reference has no distribution at all
// (one tf.Session, model/base.py:121-123).
//
// One communicator per process (one process per GPU), bootstrapped from a 128-byte ncclUniqueId that
// rank 0 publishes through the torch.distributed TCP store (parallel/native_comm.py).  Collectives run
// on a dedicated non-blocking HIP stream:
//   * enqueue: an event recorded on the caller's current stream orders the collective after the
//     kernels that produced the buffer (the backward that wrote a gradient bucket);
//   * wait:    an event recorded on the comm stream makes the caller's stream wait -- the host never
//     blocks, so bucket all-reduces overlap the rest of backward.  (Collectives are not captured into
//     hipGraphs here: the graphed train step runs its all-reduce eagerly after the replay.)
//   * the buffer is recorded on the comm stream for the caching allocator (no reuse before the
//     collective has read it).
// Linked against the librccl.so that torch itself loads (one RCCL in the process).
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include <ATen/ATen.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <torch/library.h>

namespace {

using at::Tensor;

#define INA_RCCL(call)                                                                     \
  do {                                                                                     \
    ncclResult_t r__ = (call);                                                             \
    TORCH_CHECK(r__ == ncclSuccess, "ina.comm: ", #call, " failed: ", ncclGetErrorString(r__)); \
  } while (0)
#define INA_HIP(call)                                                                      \
  do {                                                                                     \
    hipError_t e__ = (call);                                                               \
    TORCH_CHECK(e__ == hipSuccess, "ina.comm: ", #call, " failed: ", hipGetErrorString(e__)); \
  } while (0)

struct Comm {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1, device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t in = nullptr, out = nullptr;
  int64_t pending = 0;   // collectives enqueued since the last wait
};

std::mutex g_mu;
std::vector<std::unique_ptr<Comm>> g_comms;

Comm& get(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h] && g_comms[h]->comm,
              "ina.comm: invalid or destroyed communicator handle ", h);
  return *g_comms[h];
}

ncclDataType_t dtype_of(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kDouble: return ncclFloat64;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    default: TORCH_CHECK(false, "ina.comm: unsupported dtype ", t.scalar_type());
  }
}

ncclRedOp_t op_of(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  TORCH_CHECK(false, "ina.comm: unsupported reduction '", op, "'");
}

// order the comm stream after the caller's current stream; keep the buffer alive for the allocator
void enter(Comm& c, const Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "ina.comm: tensors must be contiguous GPU tensors");
  TORCH_CHECK(t.get_device() == c.device, "ina.comm: tensor on device ", t.get_device(), ", communicator on ",
              c.device);
  hipStream_t cur = c10::hip::getCurrentHIPStream(c.device).stream();
  INA_HIP(hipEventRecord(c.in, cur));
  INA_HIP(hipStreamWaitEvent(c.stream, c.in, 0));
  c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(),
                                               c10::hip::getStreamFromExternal(c.stream, c.device));
  ++c.pending;
}

}  // namespace

// 128 random bytes (CPU uint8 tensor) identifying a new communicator; rank 0 creates and publishes it
Tensor comm_unique_id() {
  ncclUniqueId id;
  INA_RCCL(ncclGetUniqueId(&id));
  auto t = at::empty({NCCL_UNIQUE_ID_BYTES}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), id.internal, NCCL_UNIQUE_ID_BYTES);
  return t;
}

int64_t comm_init(const Tensor& uid, int64_t rank, int64_t world, int64_t device) {
  TORCH_CHECK(uid.device().is_cpu() && uid.scalar_type() == at::kByte && uid.numel() == NCCL_UNIQUE_ID_BYTES,
              "ina.comm_init: uid must be the 128-byte CPU uint8 tensor of comm_unique_id()");
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "ina.comm_init: bad rank / world");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.contiguous().data_ptr(), NCCL_UNIQUE_ID_BYTES);
  auto c = std::make_unique<Comm>();
  c->rank = (int)rank;
  c->world = (int)world;
  c->device = (int)device;
  INA_HIP(hipSetDevice(c->device));
  INA_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  INA_HIP(hipEventCreateWithFlags(&c->in, hipEventDisableTiming));
  INA_HIP(hipEventCreateWithFlags(&c->out, hipEventDisableTiming));
  INA_RCCL(ncclCommInitRank(&c->comm, (int)world, id, (int)rank));
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(std::move(c));
  return (int64_t)g_comms.size() - 1;
}

// in-place all-reduce of t, enqueued on the comm stream (returns at once; comm_wait orders the caller)
void comm_allreduce_(int64_t h, Tensor t, const std::string& op) {
  Comm& c = get(h);
  enter(c, t);
  INA_RCCL(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dtype_of(t), op_of(op), c.comm, c.stream));
}

// several buffers as ONE grouped launch (bucketed flat gradient: fewer RCCL kernel launches)
void comm_allreduce_many_(int64_t h, std::vector<Tensor> ts, const std::string& op) {
  Comm& c = get(h);
  for (auto& t : ts) enter(c, t);
  INA_RCCL(ncclGroupStart());
  for (auto& t : ts)
    INA_RCCL(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dtype_of(t), op_of(op), c.comm,
                           c.stream));
  INA_RCCL(ncclGroupEnd());
}

void comm_broadcast_(int64_t h, Tensor t, int64_t root) {
  Comm& c = get(h);
  TORCH_CHECK(root >= 0 && root < c.world, "ina.comm_broadcast_: bad root");
  enter(c, t);
  INA_RCCL(ncclBroadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dtype_of(t), (int)root, c.comm, c.stream));
}

// make the caller's current stream wait for every collective enqueued so far (no host block)
void comm_wait(int64_t h) {
  Comm& c = get(h);
  if (c.pending == 0) return;
  INA_HIP(hipEventRecord(c.out, c.stream));
  INA_HIP(hipStreamWaitEvent(c10::hip::getCurrentHIPStream(c.device).stream(), c.out, 0));
  c.pending = 0;
}

// host-blocking: the comm stream has drained; surfaces asynchronous RCCL errors (failure detection)
void comm_sync(int64_t h) {
  Comm& c = get(h);
  INA_HIP(hipStreamSynchronize(c.stream));
  ncclResult_t async = ncclSuccess;
  INA_RCCL(ncclCommGetAsyncError(c.comm, &async));
  TORCH_CHECK(async == ncclSuccess, "ina.comm: asynchronous RCCL error: ", ncclGetErrorString(async));
}

std::vector<int64_t> comm_info(int64_t h) {
  Comm& c = get(h);
  int v = 0;
  ncclGetVersion(&v);
  return {c.rank, c.world, c.device, (int64_t)v};
}

// Destroys the RCCL communicator.  The comm stream and its two events stay alive for the rest of the
// process: buffers were recorded on that stream for the caching allocator (enter()), which records an
// event on it when such a block is freed later -- a destroyed stream there is a use-after-free at exit.
void comm_destroy(int64_t h) {
  std::unique_ptr<Comm> c;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (h < 0 || h >= (int64_t)g_comms.size() || !g_comms[h]) return;
    c = std::move(g_comms[h]);
  }
  hipStreamSynchronize(c->stream);
  ncclCommDestroy(c->comm);
  c->comm = nullptr;
  c.release();   // stream + events: process lifetime (see above)
}

TORCH_LIBRARY_FRAGMENT(ina, m) {
  m.def("comm_unique_id", &comm_unique_id);
  m.def("comm_init", &comm_init);
  m.def("comm_allreduce_", &comm_allreduce_);
  m.def("comm_allreduce_many_", &comm_allreduce_many_);
  m.def("comm_broadcast_", &comm_broadcast_);
  m.def("comm_wait", &comm_wait);
  m.def("comm_sync", &comm_sync);
  m.def("comm_info", &comm_info);
  m.def("comm_destroy", &comm_destroy);
}
