// Host-sanitizer driver for csrc/hclust.cpp (test infrastructure; built by tests/test_host_sanitizers.py with
// -fsanitize=address,undefined and, separately, -fsanitize=thread).  It runs the cophenetic / cutree C ABI the way
// nmf.r:165-177's replacement does -- nmfc_cophenetic_batch over a stack of consensus matrices on several host
// threads -- on consensus-like inputs (counts / R, so ties everywhere, plus n = 2 and 3 and a matrix of equal
// values) and checks that the threaded batch equals the one-matrix call bit for bit and that every cutree
// membership is a valid 1..k labelling.  Exit status 0: clean; the sanitizers abort on their own findings.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/nmfc.h"

namespace {

uint64_t lcg(uint64_t& s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return s >> 33;
}

// consensus of R clusterings of n samples into g groups with per-run label noise: entries are counts / R
std::vector<double> consensus(int n, int R, int g, uint64_t seed) {
  std::vector<int> base(n), lab(n);
  uint64_t s = seed;
  for (int i = 0; i < n; ++i) base[i] = (int)(lcg(s) % (uint64_t)g);
  std::vector<double> C((size_t)n * n, 0.0);
  for (int r = 0; r < R; ++r) {
    for (int i = 0; i < n; ++i) lab[i] = (lcg(s) % 5 == 0) ? (int)(lcg(s) % (uint64_t)g) : base[i];
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) C[(size_t)j * n + i] += lab[i] == lab[j];
  }
  for (double& v : C) v /= R;
  return C;
}

int check_stack(const std::vector<double>& C, int nk, int n, int nthreads) {
  std::vector<double> rho(nk), h1(n - 1), hb((size_t)nk * (n - 1));
  std::vector<int32_t> ob((size_t)nk * n), mb((size_t)nk * 2 * (n - 1)), o1(n), m1(2 * (n - 1)), mem(n);
  if (nmfc_cophenetic_batch(C.data(), nk, n, nthreads, rho.data(), ob.data(), mb.data(), hb.data()) != 0) return 1;
  for (int q = 0; q < nk; ++q) {
    const double r1 = nmfc_cophenetic(C.data() + (size_t)q * n * n, n, o1.data(), m1.data(), h1.data());
    if (!(std::memcmp(&r1, &rho[q], sizeof r1) == 0 || (std::isnan(r1) && std::isnan(rho[q])))) {
      std::printf("n %d matrix %d: batch rho differs from the single call\n", n, q);
      return 1;
    }
    if (std::memcmp(o1.data(), &ob[(size_t)q * n], n * sizeof(int32_t)) ||
        std::memcmp(m1.data(), &mb[(size_t)q * 2 * (n - 1)], 2 * (n - 1) * sizeof(int32_t)) ||
        std::memcmp(h1.data(), &hb[(size_t)q * (n - 1)], (n - 1) * sizeof(double))) {
      std::printf("n %d matrix %d: batch order / merge / height differ from the single call\n", n, q);
      return 1;
    }
    for (int k = 1; k <= n && k <= 8; ++k) {
      if (nmfc_cutree(m1.data(), n, k, mem.data()) != 0) return 1;
      std::vector<int> seen(k + 1, 0);
      for (int i = 0; i < n; ++i) {
        if (mem[i] < 1 || mem[i] > k) {
          std::printf("n %d k %d: membership %d out of range\n", n, k, mem[i]);
          return 1;
        }
        seen[mem[i]] = 1;
      }
      for (int c = 1; c <= k; ++c)
        if (!seen[c]) {
          std::printf("n %d k %d: cluster %d empty\n", n, k, c);
          return 1;
        }
    }
  }
  return 0;
}

}  // namespace

int main() {
  const int sizes[] = {2, 3, 17, 64, 200};
  for (int n : sizes) {
    const int nk = 9;
    std::vector<double> C;
    for (int q = 0; q < nk; ++q) {
      std::vector<double> one = consensus(n, q < 2 ? 1 : 25 + 10 * q, 2 + q % 4, 1000 + 17 * n + q);
      C.insert(C.end(), one.begin(), one.end());
    }
    if (check_stack(C, nk, n, 4)) return 1;
  }
  // every pair tied: a constant consensus matrix (zero-variance distances: rho is NaN, the tree is still built)
  std::vector<double> flat((size_t)3 * 40 * 40, 0.5);
  if (check_stack(flat, 3, 40, 3)) return 1;
  // argument checks answer without touching memory
  if (nmfc_cophenetic_batch(nullptr, 1, 10, 1, nullptr, nullptr, nullptr, nullptr) != -1) return 1;
  if (nmfc_cutree(nullptr, 5, 6, nullptr) != -1) return 1;
  std::printf("hclust driver ok\n");
  return 0;
}
