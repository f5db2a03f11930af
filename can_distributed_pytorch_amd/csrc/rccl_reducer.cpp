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

#include "bucket_schedule.h"

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <utility>
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

// The communicator is created NON-blocking (ncclConfig_t.blocking = 0) so that its
// initialisation is bounded: a rank whose peers never join (one rank failed
// before or inside its own init) polls ncclCommGetAsyncError until init_timeout_s,
// then aborts the half-made communicator and throws — every rank gets back to
// Python, where parallel/reducer.py agrees over the torch process group on
// falling back together.  In non-blocking mode any RCCL call may return
// ncclInProgress (e.g. the first collective's lazy connection setup): call()
// polls the communicator until that completes (bounded too) before the next call.
class RcclComm {
 public:
  RcclComm(int rank, int world, const std::string& uid, int device, double init_timeout_s,
           double coll_timeout_s = 120.0)
      : rank_(rank), world_(world), device_(device), timeout_(init_timeout_s), coll_timeout_(coll_timeout_s) {
    if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad ncclUniqueId size");
    ncclUniqueId id;
    memcpy(&id, uid.data(), sizeof(id));
    hip_check(hipSetDevice(device), "hipSetDevice");
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&comm_, world, id, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
      if (comm_) ncclCommAbort(comm_);
      comm_ = nullptr;
      nccl_check(r, "ncclCommInitRankConfig");
    }
    try {
      settle("ncclCommInitRankConfig", timeout_);
    } catch (...) {
      if (comm_) ncclCommAbort(comm_);
      comm_ = nullptr;
      throw;
    }
  }
  // Non-blocking communicator: finalize (flushes outstanding work) may return ncclInProgress, so it is settled with
  // a bound before the destroy; a finalize that fails or does not settle in time aborts instead of hanging the
  // process at exit.
  ~RcclComm() {
    if (!comm_) return;
    try {
      ncclResult_t r = ncclCommFinalize(comm_);
      if (r == ncclInProgress) settle("ncclCommFinalize", coll_timeout_);
      else nccl_check(r, "ncclCommFinalize");
      ncclCommDestroy(comm_);
    } catch (...) {
      ncclCommAbort(comm_);
    }
    comm_ = nullptr;
  }
  // Every RCCL call on this communicator goes through here: ncclInProgress is settled (bounded by the collective
  // timeout, much shorter than the init deadline), anything else thrown.
  void call(ncclResult_t r, const char* what) {
    if (r == ncclInProgress) {
      settle(what, coll_timeout_);
      return;
    }
    nccl_check(r, what);
  }
  void allreduce(uintptr_t ptr, size_t count, int dtype, int op, uintptr_t stream) {
    call(ncclAllReduce((const void*)ptr, (void*)ptr, count, to_dtype(dtype), to_op(op), comm_, (hipStream_t)stream),
         "ncclAllReduce");
  }
  void broadcast(uintptr_t ptr, size_t count, int dtype, int root, uintptr_t stream) {
    call(ncclBroadcast((const void*)ptr, (void*)ptr, count, to_dtype(dtype), root, comm_, (hipStream_t)stream),
         "ncclBroadcast");
  }
  void allgather(uintptr_t send, uintptr_t recv, size_t count, int dtype, uintptr_t stream) {
    call(ncclAllGather((const void*)send, (void*)recv, count, to_dtype(dtype), comm_, (hipStream_t)stream),
         "ncclAllGather");
  }
  void reduce_scatter(uintptr_t send, uintptr_t recv, size_t count, int dtype, int op, uintptr_t stream) {
    call(ncclReduceScatter((const void*)send, (void*)recv, count, to_dtype(dtype), to_op(op), comm_,
                           (hipStream_t)stream),
         "ncclReduceScatter");
  }
  // "" while healthy: ncclInProgress (a non-blocking call still settling) is not an error
  std::string async_error() {
    if (!comm_) return "communicator aborted";
    ncclResult_t r = ncclSuccess;
    ncclCommGetAsyncError(comm_, &r);
    return (r == ncclSuccess || r == ncclInProgress) ? std::string() : std::string(ncclGetErrorString(r));
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
  // Poll the communicator's state until it leaves ncclInProgress; bounded by `timeout`.
  void settle(const char* what, double timeout) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      ncclResult_t st = ncclSuccess;
      nccl_check(ncclCommGetAsyncError(comm_, &st), "ncclCommGetAsyncError");
      if (st != ncclInProgress) {
        nccl_check(st, what);
        return;
      }
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout)
        throw std::runtime_error(std::string(what) + ": timed out after " + std::to_string(timeout) +
                                 " s (did every rank join?)");
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  }
  ncclComm_t comm_ = nullptr;
  int rank_, world_, device_;
  double timeout_, coll_timeout_;
};

// Bucketed gradient all-reduce over RCCL.  The readiness logic lives in
// BucketSchedule (bucket_schedule.h, shared with the CPU fake-cluster
// transport below); this class only turns its decisions into stream work:
//   * mark_ready(params, stream): the producing stream records one event per
//     touched bucket (per (bucket, producer stream) slot, so a later mark on
//     the same stream supersedes an earlier one);
//   * a complete bucket: the comm stream waits on the events of EVERY producer
//     stream of that bucket (compute stream and/or weight-gradient side
//     stream), then ncclAllReduce(sum) in place on the arena slice;
//   * finish(): launches incomplete buckets, joins the comm stream into the
//     caller's stream with one event.  No host synchronisation anywhere.
class BucketReducer {
 public:
  // offsets/counts in ELEMENTS of the fp32 arena; param_bucket[i] = bucket of
  // parameter i (or -1 = not reduced).
  BucketReducer(RcclComm& comm, uintptr_t arena, std::vector<size_t> offsets, std::vector<size_t> counts,
                std::vector<int> param_bucket, int priority)
      : comm_(comm), arena_((float*)arena), off_(std::move(offsets)), cnt_(std::move(counts)),
        sched_(std::move(param_bucket), (int)off_.size()) {
    if (cnt_.size() != off_.size()) throw std::runtime_error("BucketReducer: offsets/counts size mismatch");
    const int nb = (int)off_.size();
    ev_.resize((size_t)nb * BucketSchedule::kMaxStreams);
    for (auto& e : ev_) hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&done_, hipEventDisableTiming), "hipEventCreate");
    int lo = 0, hi = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "priority range");
    hip_check(hipStreamCreateWithPriority(&comm_stream_, hipStreamNonBlocking, priority ? hi : lo), "stream");
  }
  ~BucketReducer() {
    for (auto& e : ev_) hipEventDestroy(e);
    for (auto& e : tev_) hipEventDestroy(e);
    hipEventDestroy(done_);
    hipStreamDestroy(comm_stream_);
  }
  // Per-bucket timing (diagnostics, off by default and never inside a captured step): timing-enabled events
  //   t_begin (compute stream at begin()), per bucket: ready = each producer stream's mark event, start / end
  //   around the all-reduce on the comm stream, and t_bwd (compute stream at finish(), every gradient written).
  // timings() turns them into milliseconds relative to t_begin; it synchronises on the events.
  void set_timing(bool on) {
    if (on && tev_.empty()) {
      const int nb = (int)off_.size();
      tev_.resize((size_t)nb * (BucketSchedule::kMaxStreams + 2) + 2);
      for (auto& e : tev_) hip_check(hipEventCreate(&e), "hipEventCreate(timing)");
    }
    timing_ = on;
  }
  void begin(uintptr_t stream) {
    sched_.begin();
    launched_.clear();
    if (timing_) {
      nready_.assign(off_.size(), 0);
      hip_check(hipEventRecord(tev_[tbegin()], (hipStream_t)stream), "record t_begin");
    }
  }
  // Returns the number of buckets launched by this call.
  int mark_ready(const std::vector<int>& params, uintptr_t stream) {
    std::vector<int> touched;
    const std::vector<int> ready = sched_.mark(params, (uint64_t)stream, &touched);
    for (int b : touched) {
      const int slot = sched_.slot_of(b, (uint64_t)stream);
      hip_check(hipEventRecord(ev_[(size_t)b * BucketSchedule::kMaxStreams + slot], (hipStream_t)stream),
                "record bucket");
      if (timing_) {
        hip_check(hipEventRecord(tev_[tready(b, slot)], (hipStream_t)stream), "record t_ready");
        nready_[b] = std::max(nready_[b], slot + 1);
      }
    }
    for (int b : ready) launch(b);
    return (int)ready.size();
  }
  void finish(uintptr_t compute_stream) {
    if (timing_) hip_check(hipEventRecord(tev_[tbwd()], (hipStream_t)compute_stream), "record t_bwd");
    for (int b : sched_.finish()) launch(b);
    hip_check(hipEventRecord(done_, comm_stream_), "record done");
    hip_check(hipStreamWaitEvent((hipStream_t)compute_stream, done_, 0), "wait done");
  }
  // [(bucket, ready_ms, start_ms, end_ms)] of the last timed step (ms after begin()) and the backward end (ms):
  // ready = the last producer of the bucket done, start/end = its all-reduce on the comm stream.
  std::pair<std::vector<std::tuple<int, double, double, double>>, double> timings() {
    std::vector<std::tuple<int, double, double, double>> out;
    if (tev_.empty()) return {out, -1.0};
    auto ms = [&](hipEvent_t e) {
      hip_check(hipEventSynchronize(e), "event sync");
      float v = 0.f;
      hip_check(hipEventElapsedTime(&v, tev_[tbegin()], e), "elapsed");
      return (double)v;
    };
    for (int b : launched_) {
      double rdy = 0.0;
      for (int i = 0; i < nready_[b]; ++i) rdy = std::max(rdy, ms(tev_[tready(b, i)]));
      out.emplace_back(b, rdy, ms(tev_[tstart(b)]), ms(tev_[tend(b)]));
    }
    return {out, ms(tev_[tbwd()])};
  }
  uintptr_t comm_stream() const { return (uintptr_t)comm_stream_; }
  int num_buckets() const { return (int)off_.size(); }
  std::vector<int> launched() const { return launched_; }

 private:
  size_t per() const { return BucketSchedule::kMaxStreams + 2; }
  size_t tready(int b, int slot) const { return (size_t)b * per() + slot; }
  size_t tstart(int b) const { return (size_t)b * per() + BucketSchedule::kMaxStreams; }
  size_t tend(int b) const { return (size_t)b * per() + BucketSchedule::kMaxStreams + 1; }
  size_t tbegin() const { return off_.size() * per(); }
  size_t tbwd() const { return off_.size() * per() + 1; }

  void launch(int b) {
    const auto& ss = sched_.streams(b);
    for (int i = 0; i < (int)ss.size(); ++i)
      hip_check(hipStreamWaitEvent(comm_stream_, ev_[(size_t)b * BucketSchedule::kMaxStreams + i], 0), "wait bucket");
    if (timing_) hip_check(hipEventRecord(tev_[tstart(b)], comm_stream_), "record t_start");
    comm_.call(ncclAllReduce(arena_ + off_[b], arena_ + off_[b], cnt_[b], ncclFloat32, ncclSum, comm_.raw(),
                             comm_stream_),
               "bucket allreduce");
    if (timing_) hip_check(hipEventRecord(tev_[tend(b)], comm_stream_), "record t_end");
    launched_.push_back(b);
  }
  RcclComm& comm_;
  float* arena_;
  std::vector<size_t> off_, cnt_;
  BucketSchedule sched_;
  std::vector<hipEvent_t> ev_, tev_;
  std::vector<int> launched_, nready_;
  bool timing_ = false;
  hipEvent_t done_;
  hipStream_t comm_stream_;
};

// ---------------------------------------------------------------------------
// CPU fake cluster: the reducer's schedule driven by W host threads (one per
// fake rank) with a blocking in-process SUM all-reduce as the transport.  The
// collective checks that every rank issues the SAME sequence of (offset,
// count) collectives — a rank that launched buckets in another order would be
// reported as a mismatch (RCCL would hang or corrupt) — and times out instead
// of hanging.  Used by tests/test_reducer_native.py.
class FakeCluster {
 public:
  FakeCluster(int world, double timeout_s)
      : world_(world), timeout_(timeout_s), ptr_(world, nullptr), off_(world, 0), cnt_(world, 0), in_(world, 0) {
    if (world < 1) throw std::runtime_error("FakeCluster: world < 1");
  }
  void allreduce(int rank, float* base, size_t off, size_t count) {
    std::unique_lock<std::mutex> lk(mu_);
    if (!err_.empty()) throw std::runtime_error(err_);
    if (in_[rank]) throw std::runtime_error("FakeCluster: rank entered a collective twice");
    in_[rank] = 1;
    ptr_[rank] = base;
    off_[rank] = off;
    cnt_[rank] = count;
    const uint64_t gen = gen_;
    if (++arrived_ == world_) {
      for (int r = 1; r < world_; ++r)
        if (off_[r] != off_[0] || cnt_[r] != cnt_[0])
          err_ = "collective #" + std::to_string(seq_) + " mismatch: rank " + std::to_string(r) + " (" +
                 std::to_string(off_[r]) + "," + std::to_string(cnt_[r]) + ") vs rank 0 (" + std::to_string(off_[0]) +
                 "," + std::to_string(cnt_[0]) + ")";
      if (err_.empty()) {
        std::vector<double> acc(count, 0.0);
        for (int r = 0; r < world_; ++r)
          for (size_t i = 0; i < count; ++i) acc[i] += ptr_[r][off + i];
        for (int r = 0; r < world_; ++r)
          for (size_t i = 0; i < count; ++i) ptr_[r][off + i] = (float)acc[i];
      }
      arrived_ = 0;
      std::fill(in_.begin(), in_.end(), 0);
      ++seq_;
      ++gen_;
      cv_.notify_all();
    } else if (!cv_.wait_for(lk, std::chrono::duration<double>(timeout_), [&] { return gen_ != gen; })) {
      if (err_.empty())
        err_ = "collective #" + std::to_string(seq_) + " timed out: ranks issued different collective sequences";
      // the cluster stays poisoned with this FIRST error; reset the rendezvous so no later call reports a
      // stale 'entered twice' instead of it
      arrived_ = 0;
      std::fill(in_.begin(), in_.end(), 0);
      ++gen_;
      cv_.notify_all();
    }
    if (!err_.empty()) throw std::runtime_error(err_);
  }
  int collectives() {
    std::lock_guard<std::mutex> lk(mu_);
    return (int)seq_;
  }

 private:
  int world_;
  double timeout_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<float*> ptr_;
  std::vector<size_t> off_, cnt_;
  std::vector<int> in_;
  int arrived_ = 0;
  uint64_t gen_ = 0, seq_ = 0;
  std::string err_;
};

// One fake rank: BucketSchedule + FakeCluster transport over a HOST fp32
// arena.  Records, per launch, the bucket and the producer-stream tags the
// GPU reducer would have waited on.
class FakeRankReducer {
 public:
  FakeRankReducer(FakeCluster& cl, int rank, uintptr_t arena, std::vector<size_t> offsets, std::vector<size_t> counts,
                  std::vector<int> param_bucket)
      : cl_(cl), rank_(rank), arena_((float*)arena), off_(std::move(offsets)), cnt_(std::move(counts)),
        sched_(std::move(param_bucket), (int)off_.size()) {}
  void begin() {
    sched_.begin();
    log_.clear();
  }
  int mark_ready(const std::vector<int>& params, uint64_t stream) {
    const std::vector<int> ready = sched_.mark(params, stream);
    for (int b : ready) launch(b);
    return (int)ready.size();
  }
  void finish() {
    for (int b : sched_.finish()) launch(b);
  }
  std::vector<std::pair<int, std::vector<uint64_t>>> log() const { return log_; }

 private:
  void launch(int b) {
    log_.emplace_back(b, sched_.streams(b));
    cl_.allreduce(rank_, arena_, off_[b], cnt_[b]);
  }
  FakeCluster& cl_;
  int rank_;
  float* arena_;
  std::vector<size_t> off_, cnt_;
  BucketSchedule sched_;
  std::vector<std::pair<int, std::vector<uint64_t>>> log_;
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
      .def(py::init([](int rank, int world, std::string uid, int device, double init_timeout_s,
                       double coll_timeout_s) {
             return new RcclComm(rank, world, uid, device, init_timeout_s, coll_timeout_s);
           }),
           py::arg("rank"), py::arg("world"), py::arg("uid"), py::arg("device"), py::arg("init_timeout_s") = 300.0,
           py::arg("coll_timeout_s") = 120.0,
           py::call_guard<py::gil_scoped_release>())
      // collectives may settle a non-blocking call (bounded): the GIL is released meanwhile
      .def("allreduce", &RcclComm::allreduce, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &RcclComm::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("allgather", &RcclComm::allgather, py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::call_guard<py::gil_scoped_release>())
      .def("async_error", &RcclComm::async_error)
      .def("abort", &RcclComm::abort)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world);
  py::class_<BucketReducer>(m, "BucketReducer")
      .def(py::init<RcclComm&, uintptr_t, std::vector<size_t>, std::vector<size_t>, std::vector<int>, int>(),
           py::keep_alive<1, 2>())
      .def("begin", &BucketReducer::begin, py::arg("stream") = 0)
      .def("mark_ready", &BucketReducer::mark_ready, py::call_guard<py::gil_scoped_release>())
      .def("finish", &BucketReducer::finish, py::call_guard<py::gil_scoped_release>())
      .def("set_timing", &BucketReducer::set_timing)
      .def("timings", &BucketReducer::timings, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("launched", &BucketReducer::launched)
      .def_property_readonly("comm_stream", &BucketReducer::comm_stream)
      .def_property_readonly("num_buckets", &BucketReducer::num_buckets);
  py::class_<BucketSchedule>(m, "BucketSchedule")
      .def(py::init<std::vector<int>, int>())
      .def("begin", &BucketSchedule::begin)
      .def("mark", [](BucketSchedule& s, const std::vector<int>& p, uint64_t stream) { return s.mark(p, stream); })
      .def("finish", &BucketSchedule::finish)
      .def("streams", &BucketSchedule::streams)
      .def("pending", &BucketSchedule::pending)
      .def_property_readonly("num_buckets", &BucketSchedule::num_buckets);
  py::class_<FakeCluster>(m, "FakeCluster")
      .def(py::init<int, double>())
      .def_property_readonly("collectives", &FakeCluster::collectives);
  py::class_<FakeRankReducer>(m, "FakeRankReducer")
      .def(py::init<FakeCluster&, int, uintptr_t, std::vector<size_t>, std::vector<size_t>, std::vector<int>>(),
           py::keep_alive<1, 2>())
      .def("begin", &FakeRankReducer::begin)
      .def("mark_ready", &FakeRankReducer::mark_ready, py::call_guard<py::gil_scoped_release>())
      .def("finish", &FakeRankReducer::finish, py::call_guard<py::gil_scoped_release>())
      .def("log", &FakeRankReducer::log);
}
