// klf_copypool.hpp — host copy workers of the staging path (klf_stage, klf_engine.cpp).
#pragma once
#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace klf {

// Host copy workers for klf_stage: one large piece is striped over a few threads, so
// staging one stream is not bound by a single core's memcpy into page-locked memory.
// The caller copies a stripe itself and waits for the rest; several callers share the
// workers (their stripes queue up).
class CopyPool {
 public:
  explicit CopyPool(int workers) {
    for (int i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int workers() const { return (int)th_.size(); }
  void copy(uint8_t* dst, const uint8_t* src, size_t n) {
    constexpr size_t kMinStripe = 256u << 10;
    const size_t parts = std::min<size_t>((size_t)workers() + 1, n / kMinStripe);
    if (parts < 2) {
      memcpy(dst, src, n);
      return;
    }
    const size_t step = (n / parts + 4095) & ~(size_t)4095;
    Job job;
    job.left = 0;
    size_t o = step;  // stripe 0 is the caller's
    {
      std::lock_guard<std::mutex> g(mu_);
      for (; o < n; o += step) {
        q_.push_back({dst + o, src + o, std::min(step, n - o), &job});
        ++job.left;
      }
    }
    cv_.notify_all();
    memcpy(dst, src, std::min(step, n));
    std::unique_lock<std::mutex> g(job.mu);
    job.cv.wait(g, [&] { return job.left == 0; });
  }

 private:
  struct Job {
    std::mutex mu;
    std::condition_variable cv;
    int left = 0;
  };
  struct Stripe {
    uint8_t* dst;
    const uint8_t* src;
    size_t n;
    Job* job;
  };
  void loop() {
    for (;;) {
      Stripe s;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        s = q_.front();
        q_.pop_front();
      }
      memcpy(s.dst, s.src, s.n);
      // notify under the job's lock: the caller (whose stack holds the job) cannot see
      // left == 0 and return before this worker is done with the job
      std::lock_guard<std::mutex> g(s.job->mu);
      if (--s.job->left == 0) s.job->cv.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Stripe> q_;
  bool stop_ = false;
  std::vector<std::thread> th_;
};

}  // namespace klf
