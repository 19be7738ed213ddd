// tools/solobench.hip -- phase cost breakdown of k_solo_mu (csrc/solo.hip: one workgroup runs a whole nmf_mu
// restart) on the gct shape (1000 x 40): FIXED iterations, per-iteration time with phases removed, and the
// phase clock stamps of wave 0.  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/solobench.hip -o tools/solobench
#include "../nmfconsensus_amd/csrc/solo.hip"

void nmfc_set_error(const char* msg) { fprintf(stderr, "%s\n", msg); }

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                               \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

template <int NCG, int KK, int SBO = 0, int SL = 0>
void bench(int m, int n, int T, bool all = true) {
  std::vector<double> a((size_t)m * n), w((size_t)m * KK), h((size_t)KK * n);
  for (size_t i = 0; i < a.size(); ++i) a[i] = 0.05 + ((i * 7919) % 1000) / 1000.0;
  for (size_t i = 0; i < w.size(); ++i) w[i] = 0.01 + ((i * 104729) % 997) / 997.0;
  for (size_t i = 0; i < h.size(); ++i) h[i] = 0.01 + ((i * 15485863) % 991) / 991.0;
  double *dA, *dW, *dH;
  int* st;
  long long* prof;
  CK(hipMalloc(&dA, a.size() * 8));
  CK(hipMalloc(&dW, w.size() * 8));
  CK(hipMalloc(&dH, h.size() * 8));
  CK(hipMalloc(&st, 64));
  CK(hipMalloc(&prof, 64));
  CK(hipMemcpy(dA, a.data(), a.size() * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("k_solo_mu<%d, %d> (F batch %d, A steps in LDS %d) on %d x %d, %d FIXED iterations\n", NCG, KK, SBO, SL, m, n, T);
  auto run = [&](auto kern, const char* name, bool stamps) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemcpy(dW, w.data(), w.size() * 8, hipMemcpyHostToDevice));
      CK(hipMemcpy(dH, h.data(), h.size() * 8, hipMemcpyHostToDevice));
      CK(hipEventRecord(e0));
      const SoloLayout lay{m, m, KK, 1, nullptr, nullptr, nullptr, 1};
      hipLaunchKernelGGL(kern, dim3(1), dim3(64 * SOLO_W), 0, 0, dA, m, n, dW, dH, T, 0, st, KK, prof, lay);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    int hs[2];
    CK(hipMemcpy(hs, st, 8, hipMemcpyDeviceToHost));
    printf("  %-30s %8.3f ms  %7.2f us/iteration  (ran %d)\n", name, best, best * 1e3 / hs[0], hs[0]);
    if (stamps) {
      long long pc[8];
      CK(hipMemcpy(pc, prof, sizeof pc, hipMemcpyDeviceToHost));
      const char* nm[7] = {"", "G MFMA+store", "barrier 1", "sums", "H update+barriers", "stop+hhT", "F,E,W rule"};
      long long tot = 0;
      for (int i = 1; i < 7; ++i) tot += pc[i];
      printf("    wave-0 cycles per iteration:");
      for (int i = 1; i < 7; ++i) printf(" %s %lld |", nm[i], pc[i] / hs[0]);
      printf(" sum %lld\n", tot / hs[0]);
    }
  };
  run(k_solo_mu<NCG, KK, 0, SBO, SL>, "full", false);
  if (!all) {
    CK(hipFree(dA));
    CK(hipFree(dW));
    CK(hipFree(dH));
    return;
  }
  run(k_solo_mu<NCG, KK, 64>, "full, phase stamps", true);
  run(k_solo_mu<NCG, KK, 1>, "no G MFMA", false);
  run(k_solo_mu<NCG, KK, 2>, "no F/E/W", false);
  run(k_solo_mu<NCG, KK, 4>, "no h h^T", false);
  run(k_solo_mu<NCG, KK, 16>, "no partial sums", false);
  run(k_solo_mu<NCG, KK, 3>, "no G, no F", false);
  run(k_solo_mu<NCG, KK, 31>, "barriers + H update only", false);
  CK(hipFree(dA));
  CK(hipFree(dW));
  CK(hipFree(dH));
}

// k_solo8_mu (ranks 5..8) phase costs: per-iteration time with phases removed (rank kt in 5..8, W/H 8 rows)
template <int NCG, int SL>
void bench8(int m, int n, int T, int kt) {
  std::vector<double> a((size_t)m * n), w((size_t)m * 8), h((size_t)8 * n);
  for (size_t i = 0; i < a.size(); ++i) a[i] = 0.05 + ((i * 7919) % 1000) / 1000.0;
  for (size_t i = 0; i < w.size(); ++i) w[i] = 0.01 + ((i * 104729) % 997) / 997.0;
  for (size_t i = 0; i < h.size(); ++i) h[i] = 0.01 + ((i * 15485863) % 991) / 991.0;
  double *dA, *dW, *dH;
  int* st;
  CK(hipMalloc(&dA, a.size() * 8));
  CK(hipMalloc(&dW, w.size() * 8));
  CK(hipMalloc(&dH, h.size() * 8));
  CK(hipMalloc(&st, 64));
  CK(hipMemcpy(dA, a.data(), a.size() * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("k_solo8_mu<%d, %d> (A steps in LDS %d) on %d x %d, rank %d, %d FIXED iterations\n", NCG, SL, SL, m, n, kt, T);
  auto run = [&](auto kern, const char* name) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemcpy(dW, w.data(), w.size() * 8, hipMemcpyHostToDevice));
      CK(hipMemcpy(dH, h.data(), h.size() * 8, hipMemcpyHostToDevice));
      const SoloLayout lay{m, m, 8, 1, nullptr, nullptr, nullptr, 1};
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3(1), dim3(64 * SOLO_W), 0, 0, dA, m, n, dW, dH, T, 0, st, kt, lay);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    int hs[2];
    CK(hipMemcpy(hs, st, 8, hipMemcpyDeviceToHost));
    printf("  %-30s %8.3f ms  %7.2f us/iteration  (ran %d)\n", name, best, best * 1e3 / hs[0], hs[0]);
  };
  run(k_solo8_mu<NCG, SL, false, 0>, "full");
  run(k_solo8_mu<NCG, SL, false, 0, 1>, "full, one gene step per F pass");
  run(k_solo8_mu<NCG, SL, false, 0, 2>, "full, two gene steps per F pass");
  run(k_solo8_mu<NCG, SL, false, 1>, "no G MFMA");
  run(k_solo8_mu<NCG, SL, false, 2>, "no F/E/W");
  run(k_solo8_mu<NCG, SL, false, 4>, "no h h^T");
  run(k_solo8_mu<NCG, SL, false, 8>, "no stop check");
  run(k_solo8_mu<NCG, SL, false, 16>, "no wave sums");
  run(k_solo8_mu<NCG, SL, false, 32>, "no H update");
  run(k_solo8_mu<NCG, SL, false, 3>, "no G, no F");
  run(k_solo8_mu<NCG, SL, false, 63>, "barriers only");
  CK(hipFree(dA));
  CK(hipFree(dW));
  CK(hipFree(dH));
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 2000;
  if (argc > 2 && atoi(argv[2]) == 8) {   // the rank 5..8 kernel only
    bench8<10, 3>(1000, 40, T, 5);
    bench8<10, 3>(1000, 40, T, 8);
    bench8<8, 2>(1000, 32, T, 8);
    return 0;
  }
  bench<10, 2>(1000, 40, T);
  bench<8, 3>(1000, 32, T);
  bench<6, 4>(1000, 24, T);
  // the A-in-LDS kernels behind k = 4 at n > 24 and k = 3 at n > 32 (padded to 4), F batch variants
  bench<8, 4, 0, 1>(1000, 32, T);
  bench<10, 4, 0, 2>(1000, 40, T);
  bench<10, 4, 2, 2>(1000, 40, T, false);
  bench<8, 3, 4>(1000, 32, T, false);
  return 0;
}
