// tools/tailbench.hip -- per-kernel times of one MU iteration at a given number of LIVE panels (C3 shape,
// 20000 x 500), for the tile shapes / LDS ring depths the engine can pick.  The tail of a REF_COMPAT sweep
// (a few restarts still running) and one GPU's shard of the 8-GPU job are small grids; this measures them
// directly.  Not part of the product.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tailbench.hip
// Usage: tailbench [R=25] [live panels list, e.g. 1,2,4,8,24]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../nmfconsensus_amd/csrc/nmfc_kernels.hpp"

using namespace nmfc;

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

template <class KF>
float timeit(KF f, int reps) {
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
  const int m = 20000, n = 500, R = argc > 1 ? atoi(argv[1]) : 25;
  std::vector<int> lives;
  {
    std::string s = argc > 2 ? argv[2] : "1,2,4,8,24";
    for (size_t p = 0; p < s.size();) {
      size_t q = s.find(',', p);
      lives.push_back(atoi(s.substr(p, q - p).c_str()));
      if (q == std::string::npos) break;
      p = q + 1;
    }
  }
  const long m_pad = (m + GT - 1) / GT * GT, n_pad = (n + BK - 1) / BK * BK, n_cols_pad = (n + 127) / 128 * 128;
  const int ngt = (int)(m_pad / GT), ntj = (int)(n_cols_pad / 128);
  const int kchunk = 2048, nsplit = (int)((m_pad + kchunk - 1) / kchunk);
  // packing of R restarts of every k = 10..2, k descending, sequential fill of 64-column panels
  std::vector<RestartInfo> ri;
  std::vector<int> pfirst;   // first restart of each panel
  int fill = PANEL, np = -1, sq = 0;
  for (int k = 10; k >= 2; --k)
    for (int r = 0; r < R; ++r) {
      if (fill + k > PANEL) {
        ++np;
        fill = 0;
        pfirst.push_back((int)ri.size());
      }
      ri.push_back({np * PANEL + fill, k, (int)ri.size(), sq});
      sq += k * k;
      fill += k;
    }
  const int total_panels = np + 1;
  pfirst.push_back((int)ri.size());
  const int maxp = (total_panels + 3) / 4 * 4;
  const long cols = (long)maxp * PANEL;
  const long sw_total = sq;
  const int nall = (int)ri.size();
  printf("tailbench C3 20000x500: R=%d -> %d restarts in %d panels; nsplit %d\n", R, nall, total_panels, nsplit);
  double *W, *Hh, *Acm, *Arm, *Gpart, *SWpart, *SH, *SHP, *Hstat;
  int *dprb, *dpre, *stop, *reason, *unch, *cls, *nst, *colact;
  RestartInfo* dri;
  ColInfo* dci;
  CK(hipMalloc(&W, sizeof(double) * cols * m_pad));
  CK(hipMalloc(&Hh, sizeof(double) * cols * n_pad));
  CK(hipMalloc(&Acm, sizeof(double) * n_cols_pad * m_pad));
  CK(hipMalloc(&Arm, sizeof(double) * m_pad * n_pad));
  CK(hipMalloc(&Gpart, sizeof(double) * nsplit * cols * n_cols_pad));
  CK(hipMalloc(&SWpart, sizeof(double) * nsplit * sw_total));
  CK(hipMalloc(&SH, sizeof(double) * sw_total));
  CK(hipMalloc(&SHP, sizeof(double) * cols * KMAX));
  CK(hipMalloc(&Hstat, sizeof(double) * nall));
  CK(hipMalloc(&colact, sizeof(int) * cols));
  CK(hipMalloc(&dci, sizeof(ColInfo) * cols));
  CK(hipMalloc(&dri, sizeof(RestartInfo) * nall));
  CK(hipMalloc(&dprb, sizeof(int) * maxp));
  CK(hipMalloc(&dpre, sizeof(int) * maxp));
  CK(hipMalloc(&stop, sizeof(int) * nall));
  CK(hipMalloc(&reason, sizeof(int) * nall));
  CK(hipMalloc(&unch, sizeof(int) * nall));
  CK(hipMalloc(&cls, sizeof(int) * nall * 512));
  CK(hipMalloc(&nst, sizeof(int)));
  {
    std::vector<double> h(std::max<long>(cols * m_pad, m_pad * n_pad));
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0.25 + (double)((i * 2654435761u) % 1000) / 1000.0;
    CK(hipMemcpy(W, h.data(), sizeof(double) * cols * m_pad, hipMemcpyHostToDevice));
    CK(hipMemcpy(Hh, h.data(), sizeof(double) * cols * n_pad, hipMemcpyHostToDevice));
    CK(hipMemcpy(Acm, h.data(), sizeof(double) * n_cols_pad * m_pad, hipMemcpyHostToDevice));
    CK(hipMemcpy(Arm, h.data(), sizeof(double) * m_pad * n_pad, hipMemcpyHostToDevice));
    std::vector<double> sp((size_t)cols * KMAX, 1e-3);
    CK(hipMemcpy(SHP, sp.data(), sizeof(double) * sp.size(), hipMemcpyHostToDevice));
  }
  // K-blocked copy of Acm: Ablk[kb][row][16] (one 16-gene block of every sample row contiguous)
  double* Ablk;
  CK(hipMalloc(&Ablk, sizeof(double) * n_cols_pad * m_pad));
  {
    std::vector<double> a((size_t)n_cols_pad * m_pad), b(a.size());
    CK(hipMemcpy(a.data(), Acm, sizeof(double) * a.size(), hipMemcpyDeviceToHost));
    for (long r = 0; r < n_cols_pad; ++r)
      for (long k = 0; k < m_pad; ++k) b[(size_t)(k / 16) * n_cols_pad * 16 + r * 16 + (k % 16)] = a[(size_t)r * m_pad + k];
    CK(hipMemcpy(Ablk, b.data(), sizeof(double) * b.size(), hipMemcpyHostToDevice));
  }
  CK(hipMemset(SWpart, 0, sizeof(double) * nsplit * sw_total));
  CK(hipMemset(unch, 0, sizeof(int) * nall));
  CK(hipMemset(cls, 0, sizeof(int) * nall * 512));
  CK(hipMemset(nst, 0, sizeof(int)));
  const long g_ld = n_cols_pad;
  const int reps = 20;
  for (int live : lives) {
    // live < 0: only the first -live restarts of panel 0 run (the end of a sweep: narrow forms apply)
    const int only = live < 0 ? -live : 0;
    live = live < 0 ? 1 : std::min(live, total_panels);
    const int npanels = (live + 3) / 4 * 4;
    const int nlive = only ? only : pfirst[live];   // restarts still running
    std::vector<ColInfo> ci((size_t)npanels * PANEL, ColInfo{0, 0, 0, 0});
    std::vector<int> prb(npanels), pre(npanels), ca((size_t)npanels * PANEL, 0), st(nall, 1);
    double useful = 0;
    for (int p = 0; p < npanels; ++p) {
      prb[p] = p < live ? pfirst[p] : nlive;
      pre[p] = p < live ? std::min(pfirst[p + 1], nlive) : nlive;
    }
    for (int q = 0; q < nlive; ++q) {
      const RestartInfo& r = ri[q];
      st[q] = 0;
      useful += 2.0 * m * n * r.k + 2.0 * m * r.k * r.k;
      for (int a = 0; a < r.k; ++a) {
        ci[r.col0 + a] = ColInfo{r.sq_off, r.col0 % PANEL, r.k, r.rid};
        ca[r.col0 + a] = 1;
      }
    }
    CK(hipMemcpy(dci, ci.data(), sizeof(ColInfo) * ci.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(colact, ca.data(), sizeof(int) * ca.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dprb, prb.data(), sizeof(int) * npanels, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpre, pre.data(), sizeof(int) * npanels, hipMemcpyHostToDevice));
    CK(hipMemcpy(stop, st.data(), sizeof(int) * nall, hipMemcpyHostToDevice));
    CK(hipMemcpy(dri, ri.data(), sizeof(RestartInfo) * nall, hipMemcpyHostToDevice));
    const long g_split = (long)npanels * PANEL * g_ld;
    printf("\n== %d live panels (%d restarts), %d panels launched, useful %.3e flop per contraction\n", live, nlive,
           npanels, useful);
#define WTA_ARGS                                                                                              \
  W, Acm, m_pad, ng, ntw, nsplit, kchunk, dprb, dpre, dri, dci, stop, Gpart, g_ld, g_split, SWpart, sw_total
#define WTA_ARGS_B                                                                                            \
  W, Ablk, m_pad, ng, ntw, nsplit, kchunk, dprb, dpre, dri, dci, stop, Gpart, g_ld, g_split, SWpart, sw_total
    auto report = [&](const char* name, float ms) {
      printf("  %-28s %8.4f ms  %6.1f TF\n", name, ms, useful / ms / 1e9);
    };
    {
      int ng = npanels, ntw = 4 * ntj;
      report("wta2 tiny 1x32 nbuf3", timeit([&] {
               hipLaunchKernelGGL((k_wta2<1, 32, 4, 1, 1, 3>), dim3(nsplit * ng * ntw), dim3(256), 0, 0, WTA_ARGS);
             }, reps));
      report("wta2 tiny 1x32 nbuf5", timeit([&] {
               hipLaunchKernelGGL((k_wta2<1, 32, 4, 1, 1, 5>), dim3(nsplit * ng * ntw), dim3(256), 0, 0, WTA_ARGS);
             }, reps));
      report("wta2 tiny 1x32 nbuf8", timeit([&] {
               hipLaunchKernelGGL((k_wta2<1, 32, 4, 1, 1, 8>), dim3(nsplit * ng * ntw), dim3(256), 0, 0, WTA_ARGS);
             }, reps));
      {   // 1-panel tiles with the Gram in workgroups of their own (the engine's tail form)
        const int ntg = ntw + 3;
        report("GIT wta2 tiny 1x32 nbuf3", timeit([&] {
                 hipLaunchKernelGGL((k_wta2<1, 32, 4, 1, 1, 3, 1, true, true, true>), dim3(nsplit * ng * ntg), dim3(256), 0, 0,
                                    W, Ablk, m_pad, ng, ntw, nsplit, kchunk, dprb, dpre, dri, dci, stop, Gpart, g_ld, g_split,
                                    SWpart, sw_total);
               }, reps));
        report("GIT wta2 tiny 1x32 nbuf8", timeit([&] {
                 hipLaunchKernelGGL((k_wta2<1, 32, 4, 1, 1, 8, 1, true, true, true>), dim3(nsplit * ng * ntg), dim3(256), 0, 0,
                                    W, Ablk, m_pad, ng, ntw, nsplit, kchunk, dprb, dpre, dri, dci, stop, Gpart, g_ld, g_split,
                                    SWpart, sw_total);
               }, reps));
        const int ntw2 = 2 * ntj, ntg2 = ntw2 + 3;
        report("GIT wta2 small 1x64 nbuf3", timeit([&] {
                 hipLaunchKernelGGL((k_wta2<1, 64, 2, 2, 1, 3, 1, true, true, true>), dim3(nsplit * ng * ntg2), dim3(256), 0, 0,
                                    W, Ablk, m_pad, ng, ntw2, nsplit, kchunk, dprb, dpre, dri, dci, stop, Gpart, g_ld, g_split,
                                    SWpart, sw_total);
               }, reps));
      }
      report("BLK wta2 tiny 1x32 nbuf3", timeit([&] {
               hipLaunchKernelGGL((k_wta2<1, 32, 4, 1, 1, 3, 1, true>), dim3(nsplit * ng * ntw), dim3(256), 0, 0, WTA_ARGS_B);
             }, reps));
      report("BLK wta2 tiny 1x32 nbuf5", timeit([&] {
               hipLaunchKernelGGL((k_wta2<1, 32, 4, 1, 1, 5, 1, true>), dim3(nsplit * ng * ntw), dim3(256), 0, 0, WTA_ARGS_B);
             }, reps));
      report("BLK wta2 tiny 1x32 nbuf8", timeit([&] {
               hipLaunchKernelGGL((k_wta2<1, 32, 4, 1, 1, 8, 1, true>), dim3(nsplit * ng * ntw), dim3(256), 0, 0, WTA_ARGS_B);
             }, reps));
      {   // bit-identity of the blocked-A form
        const size_t ng_ = (size_t)nsplit * g_split;
        std::vector<double> g1(ng_), g2(ng_);
        hipLaunchKernelGGL((k_wta2<1, 32, 4, 1, 1, 3>), dim3(nsplit * ng * ntw), dim3(256), 0, 0, WTA_ARGS);
        CK(hipMemcpy(g1.data(), Gpart, ng_ * 8, hipMemcpyDeviceToHost));
        CK(hipMemset(Gpart, 0, ng_ * 8));
        hipLaunchKernelGGL((k_wta2<1, 32, 4, 1, 1, 3, 1, true>), dim3(nsplit * ng * ntw), dim3(256), 0, 0, WTA_ARGS_B);
        CK(hipMemcpy(g2.data(), Gpart, ng_ * 8, hipMemcpyDeviceToHost));
        size_t diff = 0;
        for (size_t i = 0; i < ng_; ++i) diff += g1[i] != g2[i];
        printf("  blocked-A vs row A: %zu of %zu G partial entries differ\n", diff, ng_);
      }
      ntw = 2 * ntj;
      report("BLK wta2 small 1x64 nbuf3", timeit([&] {
               hipLaunchKernelGGL((k_wta2<1, 64, 2, 2, 1, 3, 1, true>), dim3(nsplit * ng * ntw), dim3(256), 0, 0, WTA_ARGS_B);
             }, reps));
      report("wta2 small 1x64 nbuf3", timeit([&] {
               hipLaunchKernelGGL((k_wta2<1, 64, 2, 2, 1, 3>), dim3(nsplit * ng * ntw), dim3(256), 0, 0, WTA_ARGS);
             }, reps));
      report("wta2 small 1x64 nbuf5", timeit([&] {
               hipLaunchKernelGGL((k_wta2<1, 64, 2, 2, 1, 5>), dim3(nsplit * ng * ntw), dim3(256), 0, 0, WTA_ARGS);
             }, reps));
      ng = npanels / 2;
      ntw = ntj;
      report("wta2 mid 2x128 nbuf3", timeit([&] {
               hipLaunchKernelGGL((k_wta2<2, 128, 4, 2, 1, 3>), dim3(nsplit * ng * ntw), dim3(512), 0, 0, WTA_ARGS);
             }, reps));
      report("wta2 mid 2x128 nbuf4", timeit([&] {
               hipLaunchKernelGGL((k_wta2<2, 128, 4, 2, 1, 4>), dim3(nsplit * ng * ntw), dim3(512), 0, 0, WTA_ARGS);
             }, reps));
      report("BLK wta2 mid 2x128 nbuf3", timeit([&] {
               hipLaunchKernelGGL((k_wta2<2, 128, 4, 2, 1, 3, 1, true>), dim3(nsplit * ng * ntw), dim3(512), 0, 0, WTA_ARGS_B);
             }, reps));
      ng = npanels / 4;
      report("wta2 big 4x128 nbuf3", timeit([&] {
               hipLaunchKernelGGL((k_wta2<4, 128, 4, 2, 1, 3>), dim3(nsplit * ng * ntw), dim3(512), 0, 0, WTA_ARGS);
             }, reps));
      report("BLK wta2 big 4x128 nbuf3", timeit([&] {
               hipLaunchKernelGGL((k_wta2<4, 128, 4, 2, 1, 3, 1, true>), dim3(nsplit * ng * ntw), dim3(512), 0, 0, WTA_ARGS_B);
             }, reps));
    }
    if (only && ri[nlive - 1].col0 + ri[nlive - 1].k <= 16) {   // narrow forms: live columns 0..15
      const int ntq = (int)(n_cols_pad / 16);
      report("wta narrow 16x16 nbuf4", timeit([&] {
               hipLaunchKernelGGL((k_wta_narrow<16, 4>), dim3(nsplit * (ntq + 1)), dim3(64), 0, 0, W, Acm, m_pad, ntq, nsplit,
                                  kchunk, 1, dci, Gpart, g_ld, g_split, SWpart, sw_total);
             }, reps));
      report("wta narrow 16x16 nbuf8", timeit([&] {
               hipLaunchKernelGGL((k_wta_narrow<16, 8>), dim3(nsplit * (ntq + 1)), dim3(64), 0, 0, W, Acm, m_pad, ntq, nsplit,
                                  kchunk, 1, dci, Gpart, g_ld, g_split, SWpart, sw_total);
             }, reps));
      report("BLK wta narrow 16x16 nbuf8", timeit([&] {
               hipLaunchKernelGGL((k_wta_narrow<16, 8, true>), dim3(nsplit * (ntq + 1)), dim3(64), 0, 0, W, Ablk, m_pad, ntq, nsplit,
                                  kchunk, 1, dci, Gpart, g_ld, g_split, SWpart, sw_total);
             }, reps));
      report("BLK wta narrow 16x16 nbuf16", timeit([&] {
               hipLaunchKernelGGL((k_wta_narrow<16, 16, true>), dim3(nsplit * (ntq + 1)), dim3(64), 0, 0, W, Ablk, m_pad, ntq, nsplit,
                                  kchunk, 1, dci, Gpart, g_ld, g_split, SWpart, sw_total);
             }, reps));
      report("wta narrow 16x16 nbuf16", timeit([&] {
               hipLaunchKernelGGL((k_wta_narrow<16, 16>), dim3(nsplit * (ntq + 1)), dim3(64), 0, 0, W, Acm, m_pad, ntq, nsplit,
                                  kchunk, 1, dci, Gpart, g_ld, g_split, SWpart, sw_total);
             }, reps));
      report("wta narrow 16x32 nbuf6", timeit([&] {
               hipLaunchKernelGGL((k_wta_narrow<32, 6>), dim3(nsplit * (ntq / 2 + 1)), dim3(64), 0, 0, W, Acm, m_pad, ntq / 2,
                                  nsplit, kchunk, 1, dci, Gpart, g_ld, g_split, SWpart, sw_total);
             }, reps));
    }
    report("hupdate", timeit([&] {
             hipLaunchKernelGGL(k_hupdate<>, dim3(nlive), dim3(NTH), 0, 0, 1, 1000000, STOP_FIXED, dri, n, n_pad, Gpart,
                                g_ld, g_split, nsplit, nsplit, SWpart, sw_total, Hh, SH, stop, reason, unch, cls, (long)512, nst,
                                SHP, colact, Hstat);
           }, reps));
    CK(hipMemcpy(colact, ca.data(), sizeof(int) * ca.size(), hipMemcpyHostToDevice));   // hupdate stamped iter 1
#define AHTW_ARGS(NGT) 1, Hh, n_pad, Arm, m_pad, W, SHP, dci, colact, npanels, NGT
    report("ahtw4 64 nbuf3", timeit([&] {
             hipLaunchKernelGGL((k_ahtw4<64, 3>), dim3(npanels * 2 * ngt), dim3(256), 0, 0, AHTW_ARGS(2 * ngt));
           }, reps));
    report("ahtw4 64 nbuf4", timeit([&] {
             hipLaunchKernelGGL((k_ahtw4<64, 4>), dim3(npanels * 2 * ngt), dim3(256), 0, 0, AHTW_ARGS(2 * ngt));
           }, reps));
    report("ahtw4 64 nbuf6", timeit([&] {
             hipLaunchKernelGGL((k_ahtw4<64, 6>), dim3(npanels * 2 * ngt), dim3(256), 0, 0, AHTW_ARGS(2 * ngt));
           }, reps));
    report("ahtw4 128 nbuf3", timeit([&] {
             hipLaunchKernelGGL((k_ahtw4<128, 3>), dim3(npanels * ngt), dim3(256), 0, 0, AHTW_ARGS(ngt));
           }, reps));
    report("ahtw4 128 nbuf4", timeit([&] {
             hipLaunchKernelGGL((k_ahtw4<128, 4>), dim3(npanels * ngt), dim3(256), 0, 0, AHTW_ARGS(ngt));
           }, reps));
    if (only && ri[nlive - 1].col0 + ri[nlive - 1].k <= 16) {
      report("ahtw narrow 16x64 (2w)", timeit([&] {
               hipLaunchKernelGGL((k_ahtw4<64, 3, 1, 16, 2>), dim3(2 * ngt), dim3(128), 0, 0, 1, Hh, n_pad, Arm,
                                  m_pad, W, SHP, dci, colact, 1, 2 * ngt);
             }, reps));
      report("ahtw narrow 16x32 (2w)", timeit([&] {
               hipLaunchKernelGGL((k_ahtw4<32, 3, 1, 16, 2>), dim3(4 * ngt), dim3(128), 0, 0, 1, Hh, n_pad, Arm,
                                  m_pad, W, SHP, dci, colact, 1, 4 * ngt);
             }, reps));
      report("ahtw narrow 16x128 (2w)", timeit([&] {
               hipLaunchKernelGGL((k_ahtw4<128, 3, 1, 16, 2>), dim3(ngt), dim3(128), 0, 0, 1, Hh, n_pad, Arm,
                                  m_pad, W, SHP, dci, colact, 1, ngt);
             }, reps));
    }
    report("ahtw4 2x128 nbuf3 (8w)", timeit([&] {
             hipLaunchKernelGGL((k_ahtw4<128, 3, 2>), dim3(npanels / 2 * ngt), dim3(512), 0, 0, AHTW_ARGS(ngt));
           }, reps));
    report("ahtw4 2x128 nbuf4 (8w)", timeit([&] {
             hipLaunchKernelGGL((k_ahtw4<128, 4, 2>), dim3(npanels / 2 * ngt), dim3(512), 0, 0, AHTW_ARGS(ngt));
           }, reps));
    report("ahtw4 2x64 nbuf3 (8w)", timeit([&] {
             hipLaunchKernelGGL((k_ahtw4<64, 3, 2>), dim3(npanels / 2 * 2 * ngt), dim3(512), 0, 0, AHTW_ARGS(2 * ngt));
           }, reps));
    {   // bit-identity of the 2-panel tile against the 1-panel tile (same canonical K order)
      const size_t nw = (size_t)npanels * PANEL * m_pad;
      std::vector<double> w1(nw), w2(nw), w0(nw);
      CK(hipMemcpy(w0.data(), W, nw * 8, hipMemcpyDeviceToHost));
      hipLaunchKernelGGL((k_ahtw4<128, 3>), dim3(npanels * ngt), dim3(256), 0, 0, AHTW_ARGS(ngt));
      CK(hipMemcpy(w1.data(), W, nw * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(W, w0.data(), nw * 8, hipMemcpyHostToDevice));
      hipLaunchKernelGGL((k_ahtw4<128, 3, 2>), dim3(npanels / 2 * ngt), dim3(512), 0, 0, AHTW_ARGS(ngt));
      CK(hipMemcpy(w2.data(), W, nw * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(W, w0.data(), nw * 8, hipMemcpyHostToDevice));
      size_t diff = 0, changed = 0;
      for (size_t i = 0; i < nw; ++i) {
        diff += (w1[i] != w2[i]);
        changed += (w1[i] != w0[i]);
      }
      printf("  ahtw4 2-panel vs 1-panel: %zu of %zu W entries differ (%zu updated)\n", diff, nw, changed);
    }
  }
  printf("\ndone\n");
  return 0;
}
