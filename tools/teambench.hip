// tools/teambench.hip -- phase cost breakdown of k_team_mu (the small-shape team kernel behind the nmf_mu
// drop-in) on the gct shape (1000 x 40, P = 16 workgroups): one block with ONE restart of rank k, FIXED
// iterations, per-iteration time with phases removed.  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/teambench.hip -o tools/teambench
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
  const int m = 1000, n = 40, T = argc > 1 ? atoi(argv[1]) : 2000;
  const long m_pad = 1024, n_pad = 64, ncp = 128;
  const int P = (int)(m_pad / TEAM_ROWS);
  std::vector<double> acm(ncp * m_pad, 0.0), w(16L * m_pad, 0.0), h(16L * n_pad, 0.0);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < n; ++j) acm[j * m_pad + i] = 0.5 + ((i * 7 + j * 13) % 17) / 17.0;
  for (long c = 0; c < 16; ++c) {
    for (int i = 0; i < m; ++i) w[c * m_pad + i] = 0.1 + ((c * 31 + i) % 23) / 23.0;
    for (int j = 0; j < n; ++j) h[c * n_pad + j] = 0.1 + ((c * 17 + j) % 19) / 19.0;
  }
  double *dAcm, *dW, *dH;
  double *dG, *dSW;
  unsigned* dfl;
  long long* dprof;
  int *si, *cnt;
  SmallBlock* dB;
  CK(hipMalloc(&dAcm, acm.size() * 8));
  CK(hipMalloc(&dW, w.size() * 8));
  CK(hipMalloc(&dH, h.size() * 8));
  const size_t gb = 8L * 2 * TEAM_PMAX * 16 * 64, swb = 8L * 2 * TEAM_PMAX * 256;
  CK(hipMalloc(&dfl, 4 * TEAM_PMAX));
  CK(hipMalloc(&dG, gb));
  CK(hipMalloc(&dSW, swb));
  CK(hipMalloc(&dprof, 16 * sizeof(long long)));
  CK(hipMalloc(&si, 256));
  CK(hipMalloc(&cnt, 4 * 64));
  CK(hipMalloc(&dB, sizeof(SmallBlock)));
  CK(hipMemcpy(dAcm, acm.data(), acm.size() * 8, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int k : {2, 5, 16}) {
    SmallBlock sb{};
    sb.nr = 1;
    sb.k[0] = k;
    CK(hipMemcpy(dB, &sb, sizeof sb, hipMemcpyHostToDevice));
    printf("k_team_mu on 1000 x 40, P = %d, one restart k = %d, %d FIXED iterations\n", P, k, T);
    auto run = [&](auto kern, const char* name) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemcpy(dW, w.data(), w.size() * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(dH, h.data(), h.size() * 8, hipMemcpyHostToDevice));
        CK(hipMemset(cnt, 0, 4 * 64));
        CK(hipMemset(dfl, 0, 4 * TEAM_PMAX));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(kern, dim3(P), dim3(256), 0, 0, dB, 1, P, dAcm, m_pad, n, n_pad, dW, dH, T, STOP_REF_COMPAT,
                           si, si + 1, dG, dSW, dfl, 0u, cnt, dprof);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
      }
      int hs[3];
      CK(hipMemcpy(hs, si, 12, hipMemcpyDeviceToHost));
      printf("  %-34s %8.3f ms  %7.2f us/iteration  (ran %d)\n", name, best, best * 1e3 / hs[0], hs[0]);
    };
    run(k_team_mu<3, 0>, "full");
    {
      run(k_team_mu<3, 64>, "full, phase stamps");
      long long pc[9];
      int hs[3];
      CK(hipMemcpy(pc, dprof, sizeof pc, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hs, si, 12, hipMemcpyDeviceToHost));
      const char* nm[9] = {"", "G,W^T W MFMA+store G", "store W^T W+drain+flag", "wait flags", "sum partials",
                           "H update", "h h^T + check", "F,E,W rule+stop", "wg reload"};
      long long tot = 0;
      for (int i = 1; i < 9; ++i) tot += pc[i];
      printf("    cycles per iteration by phase (workgroup 0, shader clock):");
      for (int i = 1; i < 9; ++i) printf(" %s %lld |", nm[i], pc[i] / hs[0]);
      printf(" sum %lld\n", tot / hs[0]);
    }
    run(k_team_mu<3, 1>, "no exchange");
    run(k_team_mu<3, 2>, "no G / W^T W");
    run(k_team_mu<3, 4>, "no h h^T");
    run(k_team_mu<3, 8>, "no F / E");
    run(k_team_mu<3, 16>, "no stop check");
    run(k_team_mu<3, 30>, "exchange + H update only");
    run(k_team_mu<3, 31>, "H update + barriers only");
  }
  return 0;
}
