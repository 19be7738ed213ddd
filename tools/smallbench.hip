// tools/smallbench.hip -- phase cost breakdown of k_small_mu (the small-shape persistent MU kernel) on the
// gct shape (1000 x 40): one 16-column block (restarts k = 5, 5, 5), FIXED iterations, per-iteration time
// with phases removed.  Not part of the product.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../nmfconsensus_amd/csrc/nmfc_kernels.hpp"

using namespace nmfc;
#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                               \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

int main(int argc, char** argv) {
  const int m = 1000, n = 40, T = argc > 1 ? atoi(argv[1]) : 400, nblk = argc > 2 ? atoi(argv[2]) : 1;
  const long m_pad = 1024, n_pad = 64, ncp = 128;
  std::vector<double> arm(m_pad * n_pad, 0.0), acm(ncp * m_pad, 0.0), w(16L * nblk * m_pad, 0.0),
      h(16L * nblk * n_pad, 0.0);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < n; ++j) arm[i * n_pad + j] = acm[j * m_pad + i] = 0.5 + ((i * 7 + j * 13) % 17) / 17.0;
  for (long c = 0; c < 16L * nblk; ++c) {
    for (int i = 0; i < m; ++i) w[c * m_pad + i] = 0.1 + ((c * 31 + i) % 23) / 23.0;
    for (int j = 0; j < n; ++j) h[c * n_pad + j] = 0.1 + ((c * 17 + j) % 19) / 19.0;
  }
  std::vector<SmallBlock> blocks(nblk);
  for (int b = 0; b < nblk; ++b) {
    SmallBlock sb{};
    sb.col0 = 16 * b;
    sb.nr = 3;
    for (int q = 0; q < 3; ++q) {
      sb.rid[q] = 3 * b + q;
      sb.k[q] = 5;
      sb.lc0[q] = 5 * q;
    }
    blocks[b] = sb;
  }
  double *dArm, *dAcm, *dW, *dH;
  int *si, *sr;
  SmallBlock* dB;
  CK(hipMalloc(&dArm, arm.size() * 8));
  CK(hipMalloc(&dAcm, acm.size() * 8));
  CK(hipMalloc(&dW, w.size() * 8));
  CK(hipMalloc(&dH, h.size() * 8));
  CK(hipMalloc(&si, 4 * 3 * nblk));
  CK(hipMalloc(&sr, 4 * 3 * nblk));
  CK(hipMalloc(&dB, sizeof(SmallBlock) * nblk));
  CK(hipMemcpy(dArm, arm.data(), arm.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dAcm, acm.data(), acm.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, blocks.data(), sizeof(SmallBlock) * nblk, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](auto kern, const char* name) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemcpy(dW, w.data(), w.size() * 8, hipMemcpyHostToDevice));
      CK(hipMemcpy(dH, h.data(), h.size() * 8, hipMemcpyHostToDevice));
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(kern, dim3(nblk), dim3(256), 0, 0, dB, dArm, n_pad, dAcm, m_pad, n, n_pad, dW, dH, T,
                         STOP_FIXED, si, sr);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
    }
    printf("  %-28s %8.3f ms  %7.2f us/iteration\n", name, best, best * 1e3 / T);
  };
  printf("k_small_mu on 1000 x 40, %d blocks of 3 restarts (k = 5), %d FIXED iterations\n", nblk, T);
  run(k_small_mu<16, 3, 0>, "full");
  run(k_small_mu<16, 3, 1>, "no G / W^T W");
  run(k_small_mu<16, 3, 2>, "no H update");
  run(k_small_mu<16, 3, 4>, "no h h^T / stop");
  run(k_small_mu<16, 3, 8>, "no F / E / W update");
  run(k_small_mu<16, 3, 16>, "no E = W0 (h h^T)");
  run(k_small_mu<16, 3, 32>, "W rule -> adds");
  run(k_small_mu<16, 3, 48>, "no E, W rule -> adds");
  run(k_small_mu<16, 3, 15>, "barriers only");
  return 0;
}
