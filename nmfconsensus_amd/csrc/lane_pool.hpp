// lane_pool.hpp -- the host-side lane scheduler of the Brunet sweep (csrc/brunet.hip), kept free of HIP so that
// tests/sanitize/lane_pool_driver.cpp can run it under ThreadSanitizer on the CPU with a stub job.
//
// run_lanes(nl, njobs, job, err): nl workers (lane 0 on the calling thread, lanes 1..nl-1 on std::threads) take job
// indices 0..njobs-1 from one atomic counter; job(lane, idx) returns 0 or -1.  After the first failure no worker
// starts another job; the first failing job's message (read by `err_of` on the failing thread, because the
// library's error string is thread-local) is returned in *first_err.  Every worker is joined before return, so no
// lane outlives the call.  A job may only touch state of its own lane and the outputs of its own index; everything
// shared (the counter, the failure flag, the message) is synchronised here.
#pragma once

#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace nmfc_host {

template <class Job, class ErrOf>
int run_lanes(int nl, int njobs, Job&& job, ErrOf&& err_of, std::string* first_err) {
  if (nl < 1) nl = 1;
  std::atomic<int> next{0};
  std::atomic<int> failed{0};
  std::mutex mu;
  auto worker = [&](int l) {
    for (;;) {
      if (failed.load(std::memory_order_acquire)) break;
      const int idx = next.fetch_add(1, std::memory_order_relaxed);
      if (idx >= njobs) break;
      if (job(l, idx) != 0) {
        std::lock_guard<std::mutex> g(mu);
        if (!failed.exchange(1, std::memory_order_acq_rel) && first_err) *first_err = err_of();
        break;
      }
    }
  };
  std::vector<std::thread> th;
  th.reserve(nl > 1 ? nl - 1 : 0);
  for (int l = 1; l < nl; ++l) th.emplace_back(worker, l);
  worker(0);
  for (auto& t : th) t.join();
  return failed.load() ? -1 : 0;
}

}  // namespace nmfc_host
