// tools/kvar.hip -- where the time of the full-load MFMA kernels goes (C3 shape, every restart live): A h^T
// (k_ahtw4) with its epilogue pieces switched off (VARIANT 1: no W0 loads, 2: no E, 3: no W stores, 4: no E and
// no rule) and at n = 2000 (K four times longer: the per-tile fixed cost amortised over 4x the MFMA work), and
// W^T A (k_wta2 big) with / without its Gram chains and at other ring depths.  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kvar.hip -o tools/kvar     Usage: kvar [R=200] [reps=10]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../nmfconsensus_amd/csrc/nmfc_kernels.hpp"

using namespace nmfc;

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 200, reps = argc > 2 ? atoi(argv[2]) : 10;
  const int m = 20000;
  // packing of R restarts of every k = 10..2 as the engine packs them (engine.hip pack()): k descending, first fit
  // into 16-column blocks (no restart across a block), four blocks to a 64-column panel
  std::vector<ColInfo> ci;
  std::vector<RestartInfo> ri;
  std::vector<int> pfirst;
  int np = -1, sq = 0;
  double fk = 0, fk2 = 0;   // sum of k, k^2
  {
    std::vector<int> bfill;
    std::vector<std::vector<std::pair<int, int>>> bmem;   // (k, first column in block)
    for (int k = 10; k >= 2; --k)
      for (int r = 0; r < R; ++r) {
        size_t b = 0;
        while (b < bfill.size() && bfill[b] + k > 16) ++b;
        if (b == bfill.size()) {
          bfill.push_back(0);
          bmem.emplace_back();
        }
        bmem[b].push_back({k, bfill[b]});
        bfill[b] += k;
      }
    const int nblocks = (int)bfill.size();
    np = (nblocks + 3) / 4 - 1;
    ci.assign((size_t)(np + 1) * PANEL, ColInfo{0, 0, 0, 0});
    for (int b = 0; b < nblocks; ++b) {
      if (b % 4 == 0) pfirst.push_back((int)ri.size());
      for (auto [k, c0] : bmem[b]) {
        const int col0 = 16 * b + c0;
        ri.push_back({col0, k, (int)ri.size(), sq});
        for (int a = 0; a < k; ++a) ci[(size_t)col0 + a] = ColInfo{sq, col0 % PANEL, k, (int)ri.size() - 1};
        fk += k;
        fk2 += (double)k * k;
        sq += k * k;
      }
    }
  }
  const int live = np + 1, npanels = (live + 3) / 4 * 4;
  pfirst.push_back((int)ri.size());
  ci.resize((size_t)npanels * PANEL, ColInfo{0, 0, 0, 0});
  const long cols = (long)npanels * PANEL;
  const long m_pad = (m + GT - 1) / GT * GT;
  const int ngt = (int)(m_pad / GT);
  const int nall = (int)ri.size();
  printf("kvar: R=%d, %d restarts in %d panels (%d launched), %d gene tiles\n", R, nall, live, npanels, ngt);
  const long nmax = 2048;
  double *W, *Hh, *Arm, *Ablk, *SHP, *Gpart, *SWpart;
  int *colact, *dprb, *dpre, *stop;
  ColInfo* dci;
  RestartInfo* dri;
  const long n_cols_max = nmax;
  const int kchunk = 2048, nsplit = (int)((m_pad + kchunk - 1) / kchunk);
  CK(hipMalloc(&W, sizeof(double) * cols * m_pad));
  CK(hipMalloc(&Hh, sizeof(double) * cols * nmax));
  CK(hipMalloc(&Arm, sizeof(double) * m_pad * nmax));
  CK(hipMalloc(&Ablk, sizeof(double) * m_pad * n_cols_max));
  CK(hipMalloc(&SHP, sizeof(double) * cols * KMAX));
  CK(hipMalloc(&Gpart, sizeof(double) * nsplit * cols * n_cols_max));
  CK(hipMalloc(&SWpart, sizeof(double) * nsplit * sq));
  CK(hipMalloc(&colact, sizeof(int) * cols));
  CK(hipMalloc(&dci, sizeof(ColInfo) * cols));
  CK(hipMalloc(&dri, sizeof(RestartInfo) * nall));
  CK(hipMalloc(&dprb, sizeof(int) * npanels));
  CK(hipMalloc(&dpre, sizeof(int) * npanels));
  CK(hipMalloc(&stop, sizeof(int) * nall));
  {
    std::vector<double> h((size_t)std::max<long>(cols * m_pad, m_pad * nmax));
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0.25 + (double)((i * 2654435761u) % 1000) / 1000.0;
    CK(hipMemcpy(W, h.data(), sizeof(double) * cols * m_pad, hipMemcpyHostToDevice));
    CK(hipMemcpy(Hh, h.data(), sizeof(double) * cols * nmax, hipMemcpyHostToDevice));
    CK(hipMemcpy(Arm, h.data(), sizeof(double) * m_pad * nmax, hipMemcpyHostToDevice));
    CK(hipMemcpy(Ablk, h.data(), sizeof(double) * m_pad * n_cols_max, hipMemcpyHostToDevice));
    std::vector<double> sp((size_t)cols * KMAX, 1e-3);
    CK(hipMemcpy(SHP, sp.data(), sizeof(double) * sp.size(), hipMemcpyHostToDevice));
    std::vector<int> ca(cols);
    for (long c = 0; c < cols; ++c) ca[c] = ci[c].k ? 1 : 0;
    CK(hipMemcpy(colact, ca.data(), sizeof(int) * cols, hipMemcpyHostToDevice));
    CK(hipMemcpy(dci, ci.data(), sizeof(ColInfo) * cols, hipMemcpyHostToDevice));
    CK(hipMemcpy(dri, ri.data(), sizeof(RestartInfo) * nall, hipMemcpyHostToDevice));
    std::vector<int> prb(npanels), pre(npanels);
    for (int p = 0; p < npanels; ++p) {
      prb[p] = p < live ? pfirst[p] : nall;
      pre[p] = p < live ? pfirst[p + 1] : nall;
    }
    CK(hipMemcpy(dprb, prb.data(), sizeof(int) * npanels, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpre, pre.data(), sizeof(int) * npanels, hipMemcpyHostToDevice));
    CK(hipMemset(stop, 0, sizeof(int) * nall));
  }
  auto report = [&](const char* name, float ms, double flop) {
    printf("  %-44s %8.4f ms  %6.2f TF\n", name, ms, flop / ms / 1e9);
  };
  for (long n : {500L, 2000L}) {
    const long n_pad = (n + BK - 1) / BK * BK;
    const double flop = 2.0 * m * n * fk + 2.0 * m * fk2;   // one contraction (+ its k^2 part), every restart
    printf("\n== A h^T, n = %ld (n_pad %ld)\n", n, n_pad);
#define AH(V) \
  hipLaunchKernelGGL((k_ahtw4<V, GT, 2, 1, PANEL, 4, true>), dim3(live * ngt), dim3(256), 0, 0, 1, Hh, n_pad, Arm, m_pad, W, SHP, dci, colact, live, ngt)
    report("k_ahtw4 128 LATE (engine)", timeit([&] { AH(0); }, reps), flop);
    report("  V1 no W0 loads", timeit([&] { AH(1); }, reps), flop);
    report("  V2 no E", timeit([&] { AH(2); }, reps), flop);
    report("  V3 no W stores", timeit([&] { AH(3); }, reps), flop);
    report("  V4 no E, no rule (raw F stored)", timeit([&] { AH(4); }, reps), flop);
    report("k_ahtw4 128 nbuf3 (not LATE, 2/CU)", timeit([&] {
             hipLaunchKernelGGL((k_ahtw4<0, GT, 3, 1, PANEL, 4, false>), dim3(live * ngt), dim3(256), 0, 0, 1, Hh, n_pad, Arm,
                                m_pad, W, SHP, dci, colact, live, ngt);
           }, reps), flop);
    report("k_ahtw4 2x128 nbuf3 (8 waves)", timeit([&] {
             hipLaunchKernelGGL((k_ahtw4<0, GT, 3, 2>), dim3(npanels / 2 * ngt), dim3(512), 0, 0, 1, Hh, n_pad, Arm, m_pad, W,
                                SHP, dci, colact, npanels, ngt);
           }, reps), flop);
    const long n_cols_pad = (n + 127) / 128 * 128, g_ld = n_cols_pad, g_split = cols * g_ld;
    const int ntj = (int)(n_cols_pad / 128), ng = npanels / 4;
    printf("== W^T A, n = %ld (%d sample tiles)\n", n, ntj);
#define WA(...) hipLaunchKernelGGL((k_wta2<__VA_ARGS__>), dim3(nsplit * ng * ntj), dim3(512), 0, 0, W, Ablk, m_pad, ng, ntj, nsplit, kchunk, dprb, dpre, dri, dci, stop, Gpart, g_ld, g_split, SWpart, (long)sq)
    if (ntj >= 4) {
      report("k_wta2 big 4x128 nbuf3 (engine)", timeit([&] { WA(4, 128, 4, 2, 1, 3, 1, true); }, reps), flop);
      report("  Gram from registers (GREG)", timeit([&] { WA(4, 128, 4, 2, 1, 3, 1, true, true, false, true); }, reps), flop);
      report("  no Gram chains", timeit([&] { WA(4, 128, 4, 2, 1, 3, 1, true, false); }, reps), flop);
      report("  nbuf 2", timeit([&] { WA(4, 128, 4, 2, 1, 2, 1, true); }, reps), flop);
    } else {
      report("k_wta2 big 4x128 nbuf3 GPW2 (engine)", timeit([&] { WA(4, 128, 4, 2, 2, 3, 1, true); }, reps), flop);
    }
  }
  printf("done\n");
  return 0;
}
