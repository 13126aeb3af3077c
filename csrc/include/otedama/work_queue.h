// Bounded hand-off queue between a miner thread and a host worker (the scrypt candidate verifier): the producer
// never blocks and never grows it past `cap`; a refused item is counted (the reference counts every dropped share,
// internal/miner/worker.go:266-275), and the deepest the queue has been is kept for the stats.
#pragma once
#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <vector>

namespace otedama {

template <class T>
class BoundedWorkQueue {
 public:
  explicit BoundedWorkQueue(size_t cap) : cap_(cap) {}

  // false (and counted) when full
  bool push(T&& v) {
    std::lock_guard<std::mutex> g(mu_);
    if (q_.size() >= cap_) {
      ++refused_;
      return false;
    }
    q_.push_back(std::move(v));
    peak_ = std::max<uint64_t>(peak_, q_.size());
    cv_.notify_one();
    return true;
  }

  // Blocks until an item or stop(); false once stopped and drained.
  bool pop(T* out) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
    if (q_.empty()) return false;
    *out = std::move(q_.front());
    q_.pop_front();
    return true;
  }

  // Blocks until at least one item or stop(); then takes up to `max` items. 0 once stopped and drained.
  size_t pop_many(std::vector<T>* out, size_t max) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
    size_t n = 0;
    while (!q_.empty() && n < max) {
      out->push_back(std::move(q_.front()));
      q_.pop_front();
      ++n;
    }
    return n;
  }

  // Wake the consumer to drain and exit; keep at most `keep` items (a stopping miner bounds the work left).
  void stop(size_t keep) {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
    if (q_.size() > keep) q_.resize(keep);
    cv_.notify_all();
  }

  uint64_t refused() {
    std::lock_guard<std::mutex> g(mu_);
    return refused_;
  }
  uint64_t peak() {
    std::lock_guard<std::mutex> g(mu_);
    return peak_;
  }
  size_t size() {
    std::lock_guard<std::mutex> g(mu_);
    return q_.size();
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<T> q_;
  size_t cap_;
  uint64_t refused_ = 0, peak_ = 0;
  bool stop_ = false;
};

}  // namespace otedama
