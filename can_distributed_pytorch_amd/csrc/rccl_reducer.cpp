// Native data-parallel runtime: RCCL communicator + bucketed gradient reducer.
//
// Re-implements what the reference gets from torch.nn.parallel.
// DistributedDataParallel + ProcessGroupNCCL (train.py:121-122,
// utils/distributed_utils.py:23-28), MI355X-first:
//
//  * one RCCL communicator per process (one process per GPU), bootstrapped by
//    exchanging the 128-byte ncclUniqueId through the already-initialised
//    torch process group (or its TCPStore);
//  * gradients live in ONE flat fp32 arena laid out in gradient-READY order,
//    so every bucket is a contiguous slice: no copy-in/copy-out, the
//    all-reduce runs in place (DDP's gradient_as_bucket_view, by construction);
//  * mark_ready(param) decrements the owning bucket's counter; the bucket that
//    reaches zero records an event on the compute stream, the comm stream
//    waits on it and issues ncclAllReduce(sum) — the collective overlaps with
//    the rest of the backward (dgrad/wgrad of earlier layers);
//  * finish() joins the comm stream back into the compute stream with one
//    event (no host sync); averaging by 1/world is folded into the fused SGD
//    kernel;
//  * buckets are launched in the same static order on every rank (the
//    backward schedule is static), which RCCL requires;
//  * everything is stream-ordered and hipGraph-capturable (no host syncs).
//
// Sizing for xGMI: MI355X has 7 point-to-point links per GPU; a ring all-reduce
// is bound by one link per hop, so a few large buckets (default 25 MiB, first
// 1 MiB so the all-reduce starts early) are better than many small ones, and
// the whole 82.9 MB fp32 gradient fits 4 buckets.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace can {

static void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}
static void hip_check(hipError_t r, const char* what) {
  if (r != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(r));
}

static ncclDataType_t to_dtype(int code) {
  switch (code) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclFloat64;
    case 4: return ncclInt32;
    case 5: return ncclInt64;
  }
  throw std::runtime_error("unsupported dtype code");
}
static ncclRedOp_t to_op(int code) {
  switch (code) {
    case 0: return ncclSum;
    case 1: return ncclMax;
    case 2: return ncclMin;
    case 3: return ncclProd;
  }
  throw std::runtime_error("unsupported reduce op");
}

class RcclComm {
 public:
  RcclComm(int rank, int world, const std::string& uid, int device) : rank_(rank), world_(world), device_(device) {
    if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad ncclUniqueId size");
    ncclUniqueId id;
    memcpy(&id, uid.data(), sizeof(id));
    hip_check(hipSetDevice(device), "hipSetDevice");
    nccl_check(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
  }
  ~RcclComm() {
    if (comm_) ncclCommDestroy(comm_);
  }
  void allreduce(uintptr_t ptr, size_t count, int dtype, int op, uintptr_t stream) {
    nccl_check(ncclAllReduce((const void*)ptr, (void*)ptr, count, to_dtype(dtype), to_op(op), comm_,
                             (hipStream_t)stream),
               "ncclAllReduce");
  }
  void broadcast(uintptr_t ptr, size_t count, int dtype, int root, uintptr_t stream) {
    nccl_check(ncclBroadcast((const void*)ptr, (void*)ptr, count, to_dtype(dtype), root, comm_, (hipStream_t)stream),
               "ncclBroadcast");
  }
  void allgather(uintptr_t send, uintptr_t recv, size_t count, int dtype, uintptr_t stream) {
    nccl_check(ncclAllGather((const void*)send, (void*)recv, count, to_dtype(dtype), comm_, (hipStream_t)stream),
               "ncclAllGather");
  }
  void reduce_scatter(uintptr_t send, uintptr_t recv, size_t count, int dtype, int op, uintptr_t stream) {
    nccl_check(ncclReduceScatter((const void*)send, (void*)recv, count, to_dtype(dtype), to_op(op), comm_,
                                 (hipStream_t)stream),
               "ncclReduceScatter");
  }
  std::string async_error() {
    ncclResult_t r = ncclSuccess;
    ncclCommGetAsyncError(comm_, &r);
    return r == ncclSuccess ? std::string() : std::string(ncclGetErrorString(r));
  }
  void abort() {
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }
  ncclComm_t raw() const { return comm_; }
  int rank() const { return rank_; }
  int world() const { return world_; }

 private:
  ncclComm_t comm_ = nullptr;
  int rank_, world_, device_;
};

class BucketReducer {
 public:
  // offsets/counts in ELEMENTS of the fp32 arena; param_bucket[i] = bucket of
  // parameter i (or -1 = not reduced); bucket_params[b] = #params in bucket b.
  BucketReducer(RcclComm& comm, uintptr_t arena, std::vector<size_t> offsets, std::vector<size_t> counts,
                std::vector<int> param_bucket, int priority)
      : comm_(comm), arena_((float*)arena), off_(std::move(offsets)), cnt_(std::move(counts)),
        pbucket_(std::move(param_bucket)) {
    const int nb = (int)off_.size();
    total_.assign(nb, 0);
    for (int b : pbucket_)
      if (b >= 0) total_.at(b)++;
    pending_ = total_;
    launched_.assign(nb, 0);
    ev_.resize(nb);
    for (auto& e : ev_) hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&done_, hipEventDisableTiming), "hipEventCreate");
    int lo = 0, hi = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "priority range");
    hip_check(hipStreamCreateWithPriority(&comm_stream_, hipStreamNonBlocking, priority ? hi : lo), "stream");
  }
  ~BucketReducer() {
    for (auto& e : ev_) hipEventDestroy(e);
    hipEventDestroy(done_);
    hipStreamDestroy(comm_stream_);
  }
  void begin() {
    pending_ = total_;
    std::fill(launched_.begin(), launched_.end(), 0);
    next_ = 0;
  }
  // Returns the number of buckets launched by this call.
  int mark_ready(const std::vector<int>& params, uintptr_t compute_stream) {
    for (int p : params) {
      if (p < 0 || p >= (int)pbucket_.size()) throw std::runtime_error("mark_ready: bad param index");
      const int b = pbucket_[p];
      if (b < 0) continue;
      if (--pending_[b] < 0) throw std::runtime_error("mark_ready: parameter marked twice in one step");
    }
    // launch full buckets strictly in bucket order (identical on every rank)
    int n = 0;
    while (next_ < (int)off_.size() && pending_[next_] == 0) {
      launch(next_, (hipStream_t)compute_stream);
      ++next_;
      ++n;
    }
    return n;
  }
  void finish(uintptr_t compute_stream) {
    hipStream_t cs = (hipStream_t)compute_stream;
    while (next_ < (int)off_.size()) {  // buckets holding unused params: reduce anyway
      launch(next_, cs);
      ++next_;
    }
    hip_check(hipEventRecord(done_, comm_stream_), "record done");
    hip_check(hipStreamWaitEvent(cs, done_, 0), "wait done");
  }
  uintptr_t comm_stream() const { return (uintptr_t)comm_stream_; }
  int num_buckets() const { return (int)off_.size(); }

 private:
  void launch(int b, hipStream_t cs) {
    hip_check(hipEventRecord(ev_[b], cs), "record bucket");
    hip_check(hipStreamWaitEvent(comm_stream_, ev_[b], 0), "wait bucket");
    nccl_check(ncclAllReduce(arena_ + off_[b], arena_ + off_[b], cnt_[b], ncclFloat32, ncclSum, comm_.raw(),
                             comm_stream_),
               "bucket allreduce");
    launched_[b] = 1;
  }
  RcclComm& comm_;
  float* arena_;
  std::vector<size_t> off_, cnt_;
  std::vector<int> pbucket_, total_, pending_, launched_;
  std::vector<hipEvent_t> ev_;
  hipEvent_t done_;
  hipStream_t comm_stream_;
  int next_ = 0;
};

}  // namespace can

void register_rccl(py::module_& m) {
  using namespace can;
  m.def("rccl_unique_id", []() {
    ncclUniqueId id;
    nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return py::bytes(std::string(id.internal, sizeof(id)));
  });
  m.def("rccl_version", []() {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });
  py::class_<RcclComm>(m, "RcclComm")
      // uid arrives as std::string: converted from bytes BEFORE the GIL is
      // released (ncclCommInitRank blocks until every rank has joined)
      .def(py::init([](int rank, int world, std::string uid, int device) {
             return new RcclComm(rank, world, uid, device);
           }),
           py::call_guard<py::gil_scoped_release>())
      .def("allreduce", &RcclComm::allreduce)
      .def("broadcast", &RcclComm::broadcast)
      .def("allgather", &RcclComm::allgather)
      .def("reduce_scatter", &RcclComm::reduce_scatter)
      .def("async_error", &RcclComm::async_error)
      .def("abort", &RcclComm::abort)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world);
  py::class_<BucketReducer>(m, "BucketReducer")
      .def(py::init<RcclComm&, uintptr_t, std::vector<size_t>, std::vector<size_t>, std::vector<int>, int>(),
           py::keep_alive<1, 2>())
      .def("begin", &BucketReducer::begin)
      .def("mark_ready", &BucketReducer::mark_ready)
      .def("finish", &BucketReducer::finish)
      .def_property_readonly("comm_stream", &BucketReducer::comm_stream)
      .def_property_readonly("num_buckets", &BucketReducer::num_buckets);
}
