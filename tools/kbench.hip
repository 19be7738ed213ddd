// tools/kbench.hip -- kernel micro-benchmark on C3-shaped buffers (20000 x 500, k = 2..10 x 200
// restarts, all running).  Times the product kernels of nmfc_kernels.hpp and experimental variants
// with HIP events.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kbench.hip -o tools/kbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

#include "legacy_kernels.hpp"

using namespace nmfc;
#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);      \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

// variant: A h^T main loop only (F stored, no epilogue)
static __global__ __launch_bounds__(NT, 2) void v_ahtw_main(const double* __restrict__ H, long n_pad,
                                                            const double* __restrict__ Arm, long m_pad,
                                                            double* __restrict__ F, int npanels, int ngt) {
  __shared__ __attribute__((aligned(16))) double smem[TileW::LDS_DOUBLES];
  const int item = xcd_item(blockIdx.x, npanels * ngt);
  const int gt = item % ngt, p = item / ngt;
  TileW tl;
  tl.zero();
  tl.run(H + (long)p * PANEL * n_pad, n_pad, Arm + (long)gt * GT * n_pad, n_pad, 0, (int)n_pad, smem);
#pragma unroll
  for (int mb = 0; mb < TileW::MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < TileW::NB; ++nb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg)
        F[((long)p * PANEL + TileW::row_of(mb, reg)) * m_pad + (long)gt * GT + TileW::col_of(nb)] = tl.acc[mb][nb][reg];
}

// W^T A diagnostics: MODE 0 = compute only (LDS data reused, no loads, no barriers),
// MODE 1 = compute + LDS write + barrier (no global loads), MODE 2 = full pipeline without the Gram
template <int MODE>
static __global__ __launch_bounds__(NT) void v_wta(const double* __restrict__ W, const double* __restrict__ Acm,
                                                   long m_pad, int npairs, int ntj, int nsplit, int kchunk,
                                                   double* __restrict__ Gpart, long g_ld, long g_split) {
  __shared__ __attribute__((aligned(16))) double smem[TileH::LDS_DOUBLES];
  const int nitems = nsplit * npairs * ntj;
  const int item = xcd_item(blockIdx.x, nitems);
  const int t = item % ntj;
  const int pp = (item / ntj) % npairs;
  const int s = item / (ntj * npairs);
  const double* P = W + (long)pp * 128 * m_pad;
  const double* Q = Acm + (long)t * 128 * m_pad;
  const int kbeg = s * kchunk;
  const int kend = (int)min((long)kbeg + kchunk, m_pad);
  TileH tl;
  tl.zero();
  const int nst = (kend - kbeg) / BK;
  tl.bind(P, m_pad, Q, m_pad);
  tl.gload(kbeg);
  tl.swrite(smem);
  tl.swrite(smem + TileH::STAGE);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    if (MODE == 2 && st + 1 < nst) tl.gload(kbeg + (st + 1) * BK);
    tl.compute(smem + (st & 1) * TileH::STAGE);
    if (MODE >= 1) {
      if (st + 1 < nst) tl.swrite(smem + ((st + 1) & 1) * TileH::STAGE);
      __syncthreads();
    }
  }
  double* out = Gpart + (long)s * g_split + (long)pp * 128 * g_ld + (long)t * 128;
#pragma unroll
  for (int mb = 0; mb < TileH::MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < TileH::NB; ++nb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg)
        out[(long)TileH::row_of(mb, reg) * g_ld + TileH::col_of(nb)] = tl.acc[mb][nb][reg];
}

template <class KF>
float timeit(KF f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int m = 20000, n = 500, R = argc > 1 ? atoi(argv[1]) : 200;
  std::vector<int> ks;
  for (int k = 10; k >= 2; --k) ks.push_back(k);
  const long m_pad = (m + GT - 1) / GT * GT, n_pad = (n + BK - 1) / BK * BK, n_cols_pad = (n + 127) / 128 * 128;
  const int ngt = (int)(m_pad / GT);
  const int kchunk = 2048, nsplit = (int)((m_pad + kchunk - 1) / kchunk);
  // packing
  std::vector<RestartInfo> ri;
  std::vector<int> prb, pre;
  int fill = PANEL, np = -1, sq = 0, rid = 0;
  double useful = 0;
  for (int k : ks)
    for (int r = 0; r < R; ++r) {
      if (fill + k > PANEL) {
        ++np;
        fill = 0;
        prb.push_back((int)ri.size());
        pre.push_back((int)ri.size());
      }
      ri.push_back({np * PANEL + fill, k, rid++, sq});
      sq += k * k;
      fill += k;
      pre[np] = (int)ri.size();
      useful += 2.0 * m * n * k + 2.0 * m * k * k;
    }
  int npanels = np + 1;
  while (npanels & 3) {   // multiple of 4 (k_wta2 panel quads)
    prb.push_back((int)ri.size());
    pre.push_back((int)ri.size());
    ++npanels;
  }
  const long cols = (long)npanels * PANEL;
  const long sw_total = sq;
  const int nact = (int)ri.size();
  printf("C3 kernel bench: %d restarts, %d panels, useful flops per contraction %.3e\n", nact, npanels, useful);
  double *W, *Hh, *Acm, *Arm, *Gpart, *SWpart, *SH, *F;
  int *dprb, *dpre, *stop, *reason, *unch, *cls, *nst;
  RestartInfo* dri;
  CK(hipMalloc(&W, sizeof(double) * cols * m_pad));
  CK(hipMalloc(&Hh, sizeof(double) * cols * n_pad));
  CK(hipMalloc(&F, sizeof(double) * cols * m_pad));
  CK(hipMalloc(&Acm, sizeof(double) * n_cols_pad * m_pad));
  CK(hipMalloc(&Arm, sizeof(double) * m_pad * n_pad));
  CK(hipMalloc(&Gpart, sizeof(double) * nsplit * cols * n_cols_pad));
  CK(hipMalloc(&SWpart, sizeof(double) * nsplit * sw_total));
  ColInfo* dci;
  CK(hipMalloc(&dci, sizeof(ColInfo) * npanels * PANEL));
  {
    std::vector<ColInfo> ci((size_t)npanels * PANEL, ColInfo{0, 0, 0, 0});
    for (const RestartInfo& r : ri)
      for (int a = 0; a < r.k; ++a) ci[r.col0 + a] = ColInfo{r.sq_off, r.col0 % PANEL, r.k, r.rid};
    CK(hipMemcpy(dci, ci.data(), sizeof(ColInfo) * ci.size(), hipMemcpyHostToDevice));
  }
  CK(hipMalloc(&SH, sizeof(double) * sw_total));
  double* SHP;
  CK(hipMalloc(&SHP, sizeof(double) * cols * KMAX));
  int* colact;
  CK(hipMalloc(&colact, sizeof(int) * cols));
  {
    std::vector<int> ca(cols, 0);
    for (const RestartInfo& r : ri)
      for (int a = 0; a < r.k; ++a) ca[r.col0 + a] = 1;   // iteration 1
    CK(hipMemcpy(colact, ca.data(), sizeof(int) * cols, hipMemcpyHostToDevice));
  }
  CK(hipMalloc(&dri, sizeof(RestartInfo) * nact));
  CK(hipMalloc(&dprb, sizeof(int) * npanels));
  CK(hipMalloc(&dpre, sizeof(int) * npanels));
  CK(hipMalloc(&stop, sizeof(int) * nact));
  CK(hipMalloc(&reason, sizeof(int) * nact));
  CK(hipMalloc(&unch, sizeof(int) * nact));
  CK(hipMalloc(&cls, sizeof(int) * nact * 512));
  CK(hipMalloc(&nst, sizeof(int)));
  {
    std::vector<double> h(std::max<long>(cols * m_pad, m_pad * n_pad));
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0.25 + (double)((i * 2654435761u) % 1000) / 1000.0;
    CK(hipMemcpy(W, h.data(), sizeof(double) * cols * m_pad, hipMemcpyHostToDevice));
    CK(hipMemcpy(Hh, h.data(), sizeof(double) * cols * n_pad, hipMemcpyHostToDevice));
    CK(hipMemcpy(Acm, h.data(), sizeof(double) * n_cols_pad * m_pad, hipMemcpyHostToDevice));
    CK(hipMemcpy(Arm, h.data(), sizeof(double) * m_pad * n_pad, hipMemcpyHostToDevice));
    std::vector<double> s(sw_total, 1e-3);
    CK(hipMemcpy(SH, s.data(), sizeof(double) * sw_total, hipMemcpyHostToDevice));
    std::vector<double> sp((size_t)cols * KMAX, 0.0);
    for (const RestartInfo& r : ri)
      for (int a = 0; a < r.k; ++a)
        for (int b = 0; b < r.k; ++b) sp[(size_t)(r.col0 + a) * KMAX + b] = 1e-3;
    CK(hipMemcpy(SHP, sp.data(), sizeof(double) * sp.size(), hipMemcpyHostToDevice));
  }
  CK(hipMemcpy(dri, ri.data(), sizeof(RestartInfo) * nact, hipMemcpyHostToDevice));
  CK(hipMemcpy(dprb, prb.data(), sizeof(int) * npanels, hipMemcpyHostToDevice));
  CK(hipMemcpy(dpre, pre.data(), sizeof(int) * npanels, hipMemcpyHostToDevice));
  CK(hipMemset(stop, 0, sizeof(int) * nact));
  CK(hipMemset(SWpart, 0, sizeof(double) * nsplit * sw_total));
  const int npairs = npanels / 2, ntj = (int)(n_cols_pad / 128);
  const long g_ld = n_cols_pad, g_split = cols * g_ld;
  const int reps = 10;
  float t;
  t = timeit([&] {
    hipLaunchKernelGGL((k_wta<1, true>), dim3(nsplit * npairs * ntj), dim3(NT), 0, 0, W, Acm, m_pad, npairs, ntj, nsplit, kchunk,
                       dprb, dpre, dri, dci, stop, Gpart, g_ld, g_split, SWpart, sw_total);
  }, reps);
  printf("k_wta        %8.3f ms  %6.1f TF useful  %6.1f TF executed\n", t, useful / t / 1e9,
         2.0 * cols * m_pad * n_cols_pad / t / 1e9);
  {
    const size_t gn = (size_t)nsplit * cols * n_cols_pad, sn = (size_t)nsplit * sw_total;
    std::vector<double> g1(gn), g2(gn), s1(sn), s2(sn);
    CK(hipMemcpy(g1.data(), Gpart, gn * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(s1.data(), SWpart, sn * 8, hipMemcpyDeviceToHost));
    CK(hipMemset(Gpart, 0, gn * 8));
    CK(hipMemset(SWpart, 0, sn * 8));
    const int ngroups = npanels / 4;
    auto kw2 = [&] {
      hipLaunchKernelGGL((k_wta2<4, 128, 4, 2, 1>), dim3(nsplit * ngroups * ntj), dim3(512), 0, 0, W, Acm, m_pad, ngroups, ntj,
                         nsplit, kchunk, dprb, dpre, dri, dci, stop, Gpart, g_ld, g_split, SWpart, sw_total);
    };
    kw2();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(g2.data(), Gpart, gn * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(s2.data(), SWpart, sn * 8, hipMemcpyDeviceToHost));
    double md = 0, mx = 0, sd = 0, sx = 0;
    for (size_t i = 0; i < gn; ++i) { md = std::max(md, std::fabs(g1[i] - g2[i])); mx = std::max(mx, std::fabs(g1[i])); }
    for (size_t i = 0; i < sn; ++i) { sd = std::max(sd, std::fabs(s1[i] - s2[i])); sx = std::max(sx, std::fabs(s1[i])); }
    printf("wta2 vs wta: G max|d| %.3e (max %.3e)  Gram max|d| %.3e (max %.3e)\n", md, mx, sd, sx);
    for (int rep = 0; rep < 3; ++rep) {
      t = timeit(kw2, reps);
      printf("k_wta2 256x128 8w  %8.3f ms  %6.1f TF useful  %6.1f TF executed\n", t, useful / t / 1e9,
             2.0 * cols * m_pad * n_cols_pad / t / 1e9);
    }
  }
  {
    const double ex = 2.0 * cols * m_pad * n_cols_pad;
    t = timeit([&] {
      hipLaunchKernelGGL(v_wta<0>, dim3(nsplit * npairs * ntj), dim3(NT), 0, 0, W, Acm, m_pad, npairs, ntj, nsplit,
                         kchunk, Gpart, g_ld, g_split);
    }, reps);
    printf("wta compute-only        %8.3f ms  %6.1f TF executed\n", t, ex / t / 1e9);
    t = timeit([&] {
      hipLaunchKernelGGL(v_wta<1>, dim3(nsplit * npairs * ntj), dim3(NT), 0, 0, W, Acm, m_pad, npairs, ntj, nsplit,
                         kchunk, Gpart, g_ld, g_split);
    }, reps);
    printf("wta +lds write+barrier  %8.3f ms  %6.1f TF executed\n", t, ex / t / 1e9);
    t = timeit([&] {
      hipLaunchKernelGGL(v_wta<2>, dim3(nsplit * npairs * ntj), dim3(NT), 0, 0, W, Acm, m_pad, npairs, ntj, nsplit,
                         kchunk, Gpart, g_ld, g_split);
    }, reps);
    printf("wta full, no gram       %8.3f ms  %6.1f TF executed\n", t, ex / t / 1e9);
  }
  t = timeit([&] {
    hipLaunchKernelGGL(v_ahtw_main, dim3(npanels * ngt), dim3(NT), 0, 0, Hh, n_pad, Arm, m_pad, F, npanels, ngt);
  }, reps);
  printf("ahtw main    %8.3f ms  %6.1f TF useful  %6.1f TF executed\n", t, useful / t / 1e9,
         2.0 * cols * m_pad * n_pad / t / 1e9);
  t = timeit([&] {
    // iter = 1: all restarts live; the W update writes W in place (values stay finite)
    hipLaunchKernelGGL(k_ahtw, dim3(npanels * ngt), dim3(NT), 0, 0, 1, Hh, n_pad, Arm, m_pad, W, SH, dprb, dpre, dri,
                       dci, stop, npanels, ngt);
  }, reps);
  printf("k_ahtw       %8.3f ms  %6.1f TF useful\n", t, useful / t / 1e9);
  {
    // parity of ahtw2 vs ahtw from the same W0 (one launch each), then timing
    double* W2;
    const size_t wn = (size_t)cols * m_pad;
    CK(hipMalloc(&W2, wn * 8));
    std::vector<double> h(wn);
    for (size_t i = 0; i < wn; ++i) h[i] = 0.25 + (double)((i * 2654435761u) % 1000) / 1000.0;
    CK(hipMemcpy(W, h.data(), wn * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(W2, h.data(), wn * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_ahtw, dim3(npanels * ngt), dim3(NT), 0, 0, 1, Hh, n_pad, Arm, m_pad, W, SH, dprb, dpre, dri,
                       dci, stop, npanels, ngt);
    hipLaunchKernelGGL(k_ahtw4<0>, dim3(npanels * ngt), dim3(256), 0, 0, 1, Hh, n_pad, Arm, m_pad, W2, SHP, dci, colact,
                       npanels, ngt);
    CK(hipDeviceSynchronize());
    std::vector<double> a1(wn), a2(wn);
    CK(hipMemcpy(a1.data(), W, wn * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(a2.data(), W2, wn * 8, hipMemcpyDeviceToHost));
    double md = 0, mx = 0;
    size_t nbad = 0;
    for (size_t i = 0; i < wn; ++i) {
      const double d = std::fabs(a1[i] - a2[i]);
      md = std::max(md, d / std::max(std::fabs(a1[i]), 1e-300));
      mx = std::max(mx, std::fabs(a1[i]));
      nbad += d > 1e-12 * std::fabs(a1[i]);
    }
    printf("ahtw4 vs ahtw: W max rel diff %.3e (max %.3e), %zu entries off by >1e-12\n", md, mx, nbad);
    CK(hipFree(W2));
#define AHTW2_VAR(V, label)                                                                                  \
    t = timeit([&] {                                                                                        \
      hipLaunchKernelGGL(k_ahtw2<V>, dim3(npanels * ngt), dim3(256), 0, 0, 1, Hh, n_pad, Arm, m_pad, W, SH, dprb, \
                         dpre, dri, dci, stop, npanels, ngt);                                               \
    }, reps);                                                                                               \
    printf("k_ahtw2 %-14s %8.3f ms  %6.1f TF useful\n", label, t, useful / t / 1e9);
    AHTW2_VAR(0, "")
    AHTW2_VAR(0, "")
    AHTW2_VAR(1, "no W0 load")
    AHTW2_VAR(2, "no E")
    AHTW2_VAR(3, "no W store")
    AHTW2_VAR(4, "main only")
#define AHTW3_VAR(V, label)                                                                                  \
    t = timeit([&] {                                                                                        \
      hipLaunchKernelGGL((k_ahtw2<V, 1>), dim3(npanels * ngt), dim3(256), 0, 0, 1, Hh, n_pad, Arm, m_pad, W, SH, dprb, \
                         dpre, dri, dci, stop, npanels, ngt);                                               \
    }, reps);                                                                                               \
    printf("k_ahtw3 %-14s %8.3f ms  %6.1f TF useful\n", label, t, useful / t / 1e9);
    AHTW3_VAR(0, "")
    AHTW3_VAR(0, "")
    AHTW3_VAR(1, "no W0 load")
    AHTW3_VAR(2, "no E")
    AHTW3_VAR(4, "main only")
#define AHTW4_VAR(V, label)                                                                                  \
    t = timeit([&] {                                                                                        \
      hipLaunchKernelGGL(k_ahtw4<V>, dim3(npanels * ngt), dim3(256), 0, 0, 1, Hh, n_pad, Arm, m_pad, W, SHP, dci, colact, \
                         npanels, ngt);                                                                     \
    }, reps);                                                                                               \
    printf("k_ahtw4 %-14s %8.3f ms  %6.1f TF useful\n", label, t, useful / t / 1e9);
    AHTW4_VAR(0, "")
    AHTW4_VAR(0, "")
    AHTW4_VAR(1, "no W0 load")
    AHTW4_VAR(2, "no E")
    AHTW4_VAR(4, "main only")
  }
#define AHTW_VAR(V, label)                                                                                  \
  t = timeit([&] {                                                                                          \
    hipLaunchKernelGGL(k_ahtw_t<V>, dim3(npanels * ngt), dim3(NT), 0, 0, 1, Hh, n_pad, Arm, m_pad, W, SH, dprb, \
                       dpre, dri, dci, stop, npanels, ngt);                                              \
  }, reps);                                                                                                 \
  printf("k_ahtw %-14s %8.3f ms\n", label, t);
  AHTW_VAR(1, "no W0 load")
  AHTW_VAR(2, "no E")
  AHTW_VAR(3, "no W store")
  t = timeit([&] {
    hipLaunchKernelGGL(k_hupdate, dim3(nact), dim3(NT), 0, 0, 1, 10000, 0, dri, n, n_pad, Gpart, g_ld, g_split, nsplit,
                       SWpart, sw_total, Hh, SH, stop, reason, unch, cls, 512L, nst, SHP, colact, nullptr);
  }, reps);
  printf("k_hupdate    %8.3f ms\n", t);
  return 0;
}
