// lane_pool_driver.cpp -- the Brunet sweep's lane scheduler (csrc/lane_pool.hpp) with a stub job, for
// tests/test_host_sanitizers.py under ThreadSanitizer (and ASan + UBSan).  The stub does what br_run_k does to shared
// state: per-lane scratch that grows (Buf::ensure), a thread-local error string set on failure, per-lane iteration
// tallies, and writes into the caller's output arrays at its own job index only.  Checks: every job runs exactly
// once, outputs equal a serial run, a failing job stops the others from starting new jobs and its message is the one
// returned, and lane counts 1..8 all agree.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../nmfconsensus_amd/csrc/lane_pool.hpp"

namespace {

thread_local std::string g_err;   // as engine.hip's nmfc_set_error / nmfc_last_error

struct Lane {
  std::vector<double> scratch;   // grows like the lane's device buffers
  long long iters = 0;
  int max_it = 0;
};

int stub_job(Lane& L, int idx, int fail_at, std::vector<double>& out, std::vector<int>& ran) {
  const size_t need = 1000 + 97 * (size_t)(idx % 13);
  if (L.scratch.size() < need) L.scratch.assign(need, 0.0);
  double acc = 0.0;
  for (size_t i = 0; i < need; ++i) {
    L.scratch[i] = (double)(idx + 1) * (double)(i % 17);
    acc += L.scratch[i];
  }
  ran[idx] += 1;
  if (idx == fail_at) {
    char buf[64];
    snprintf(buf, sizeof buf, "stub job %d failed", idx);
    g_err = buf;
    return -1;
  }
  out[idx] = acc;
  const int it = 100 + idx % 7;
  L.iters += it;
  if (it > L.max_it) L.max_it = it;
  return 0;
}

}  // namespace

int main() {
  const int njobs = 57;
  std::vector<double> serial(njobs, 0.0);
  std::vector<int> ran_serial(njobs, 0);
  {
    Lane L;
    for (int i = 0; i < njobs; ++i) stub_job(L, i, -1, serial, ran_serial);
  }
  for (int rep = 0; rep < 20; ++rep) {
    for (int nl = 1; nl <= 8; ++nl) {
      std::vector<Lane> lanes(nl);
      std::vector<double> out(njobs, 0.0);
      std::vector<int> ran(njobs, 0);
      std::string err;
      const int rc = nmfc_host::run_lanes(
          nl, njobs, [&](int l, int idx) { return stub_job(lanes[l], idx, -1, out, ran); },
          [] { return g_err; }, &err);
      if (rc != 0 || !err.empty()) {
        fprintf(stderr, "nl=%d: unexpected failure rc=%d err=%s\n", nl, rc, err.c_str());
        return 1;
      }
      long long tot = 0;
      for (auto& L : lanes) tot += L.iters;
      long long tot_serial = 0;
      for (int i = 0; i < njobs; ++i) tot_serial += 100 + i % 7;
      for (int i = 0; i < njobs; ++i)
        if (ran[i] != 1 || out[i] != serial[i]) {
          fprintf(stderr, "nl=%d: job %d ran %d times, out %g vs %g\n", nl, i, ran[i], out[i], serial[i]);
          return 1;
        }
      if (tot != tot_serial) {
        fprintf(stderr, "nl=%d: iteration tally %lld vs %lld\n", nl, tot, tot_serial);
        return 1;
      }
      // a failing job: the call fails with that job's message; no job runs twice
      std::vector<Lane> lanes2(nl);
      std::vector<int> ran2(njobs, 0);
      std::vector<double> out2(njobs, 0.0);
      const int fail_at = (7 * rep + nl) % njobs;
      const int rc2 = nmfc_host::run_lanes(
          nl, njobs, [&](int l, int idx) { return stub_job(lanes2[l], idx, fail_at, out2, ran2); },
          [] { return g_err; }, &err);
      char want[64];
      snprintf(want, sizeof want, "stub job %d failed", fail_at);
      if (rc2 != -1 || err != want) {
        fprintf(stderr, "nl=%d: failure not reported (rc=%d err=%s)\n", nl, rc2, err.c_str());
        return 1;
      }
      for (int i = 0; i < njobs; ++i)
        if (ran2[i] > 1) {
          fprintf(stderr, "nl=%d: job %d ran twice after a failure\n", nl, i);
          return 1;
        }
      if (ran2[fail_at] != 1) return 1;
    }
  }
  printf("lane pool driver ok\n");
  return 0;
}
