// Concurrent queues.
//
// Parity: src/include/concurrent_queue.h: concurrent_queue (MPMC, :49-99), concurrent_quota_queue
// (bounded, :116-178) and concurrent_external_quota_queue (reserve -> push_reserved ->
// pop_without_dereserve -> dereserve, :196-272), the last one bounding in-flight LPQs in the
// hybrid merge.
#pragma once
#include <condition_variable>
#include <cstddef>
#include <deque>
#include <mutex>

namespace uda {

template <typename T>
class ConcurrentQueue {
 public:
  void push(T v) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(v));
    }
    cv_.notify_one();
  }
  T wait_and_pop() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return !q_.empty(); });
    T v = std::move(q_.front());
    q_.pop_front();
    return v;
  }
  bool try_pop(T* out) {
    std::lock_guard<std::mutex> g(mu_);
    if (q_.empty()) return false;
    *out = std::move(q_.front());
    q_.pop_front();
    return true;
  }
  size_t size() const {
    std::lock_guard<std::mutex> g(mu_);
    return q_.size();
  }
  bool empty() const { return size() == 0; }

 private:
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<T> q_;
};

// Bounded queue: push blocks while `quota` elements are queued.
template <typename T>
class QuotaQueue {
 public:
  explicit QuotaQueue(size_t quota) : quota_(quota ? quota : 1) {}
  void push(T v) {
    std::unique_lock<std::mutex> lk(mu_);
    not_full_.wait(lk, [&] { return q_.size() < quota_; });
    q_.push_back(std::move(v));
    not_empty_.notify_one();
  }
  T pop() {
    std::unique_lock<std::mutex> lk(mu_);
    not_empty_.wait(lk, [&] { return !q_.empty(); });
    T v = std::move(q_.front());
    q_.pop_front();
    not_full_.notify_one();
    return v;
  }

 private:
  size_t quota_;
  std::mutex mu_;
  std::condition_variable not_full_, not_empty_;
  std::deque<T> q_;
};

// External quota: a producer reserves a slot *before* producing (so at most `quota` items are
// being produced or waiting), the consumer releases the slot only after it finished with the item.
template <typename T>
class ExternalQuotaQueue {
 public:
  explicit ExternalQuotaQueue(size_t quota) : quota_(quota ? quota : 1) {}
  void wait_and_reserve() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return reserved_ < quota_; });
    ++reserved_;
  }
  void push_reserved(T v) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(v));
    }
    cv_.notify_all();
  }
  T wait_and_pop_without_dereserve() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return !q_.empty(); });
    T v = std::move(q_.front());
    q_.pop_front();
    return v;
  }
  void dereserve() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (reserved_) --reserved_;
    }
    cv_.notify_all();
  }
  size_t reserved() const {
    std::lock_guard<std::mutex> g(mu_);
    return reserved_;
  }

 private:
  size_t quota_;
  size_t reserved_ = 0;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<T> q_;
};

}  // namespace uda
