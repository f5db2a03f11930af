// Bucket readiness schedule of the data-parallel reducer (pure host C++, no
// HIP, no RCCL): the part of DDP's Reducer that decides WHEN a gradient
// bucket may be all-reduced (reference: torch DDP at train.py:121-122;
// SURVEY §2.4 / §2.6 N5).  Shared by
//   * BucketReducer (rccl_reducer.cpp): RCCL all-reduce on a comm stream,
//   * FakeRankReducer (rccl_reducer.cpp): CPU fake-cluster transport for the
//     multi-rank tests (tests/test_reducer_native.py),
// so the logic the GPU runs is exactly the logic the CPU tests exercise.
//
// Rules:
//   * every parameter maps to one bucket (or -1: never reduced); a bucket is
//     complete once each of its parameters has been marked once this step;
//   * complete buckets launch strictly in bucket order (the order is the same
//     on every rank, which RCCL requires — a rank whose marks arrive in a
//     different interleaving still issues the identical collective sequence);
//   * each mark carries the tag of the stream that produced the gradient (the
//     compute stream or the weight-gradient side stream).  The schedule keeps,
//     per bucket, the set of producer streams, so the transport can make the
//     collective wait on EVERY producer, not only on the stream of the last
//     mark.
#pragma once

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace can {

class BucketSchedule {
 public:
  static constexpr int kMaxStreams = 4;   // distinct producer streams per bucket

  BucketSchedule(std::vector<int> param_bucket, int nbuckets)
      : pbucket_(std::move(param_bucket)), total_(nbuckets, 0) {
    for (int b : pbucket_) {
      if (b >= nbuckets) throw std::runtime_error("BucketSchedule: bucket index out of range");
      if (b >= 0) total_[b]++;
    }
    streams_.assign(nbuckets, {});
    begin();
  }

  void begin() {
    pending_ = total_;
    next_ = 0;
    for (auto& s : streams_) s.clear();
  }

  // Marks parameters produced on `stream`.  Returns the bucket(s) this mark
  // touched (for per-mark event recording) through `touched`, and the buckets
  // that became launchable, in launch order.
  std::vector<int> mark(const std::vector<int>& params, uint64_t stream, std::vector<int>* touched = nullptr) {
    for (int p : params) {
      if (p < 0 || p >= (int)pbucket_.size()) throw std::runtime_error("mark_ready: bad param index " + std::to_string(p));
      const int b = pbucket_[p];
      if (b < 0) continue;
      if (b < next_) throw std::runtime_error("mark_ready: parameter " + std::to_string(p) + " of an already launched bucket");
      if (--pending_[b] < 0) throw std::runtime_error("mark_ready: parameter " + std::to_string(p) + " marked twice in one step");
      auto& ss = streams_[b];
      const bool fresh = std::find(ss.begin(), ss.end(), stream) == ss.end();
      if (fresh) {
        if ((int)ss.size() >= kMaxStreams) throw std::runtime_error("mark_ready: too many producer streams for one bucket");
        ss.push_back(stream);
      }
      if (touched && std::find(touched->begin(), touched->end(), b) == touched->end()) touched->push_back(b);
    }
    std::vector<int> ready;
    while (next_ < (int)total_.size() && pending_[next_] == 0) ready.push_back(next_++);
    return ready;
  }

  // End of backward: buckets still incomplete (parameters that got no gradient
  // this step) are launched anyway, in order, like DDP without
  // find_unused_parameters (the stale slots are reduced as they are).
  std::vector<int> finish() {
    std::vector<int> rest;
    while (next_ < (int)total_.size()) rest.push_back(next_++);
    return rest;
  }

  int slot_of(int bucket, uint64_t stream) const {
    const auto& ss = streams_.at(bucket);
    for (int i = 0; i < (int)ss.size(); ++i)
      if (ss[i] == stream) return i;
    return -1;
  }
  const std::vector<uint64_t>& streams(int bucket) const { return streams_.at(bucket); }
  int pending(int bucket) const { return pending_.at(bucket); }
  int num_buckets() const { return (int)total_.size(); }
  int next() const { return next_; }

 private:
  std::vector<int> pbucket_, total_, pending_;
  std::vector<std::vector<uint64_t>> streams_;
  int next_ = 0;
};

}  // namespace can
