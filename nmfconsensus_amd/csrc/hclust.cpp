// hclust.cpp -- host side of the cophenetic step (nmf.r:165-177):
//   dist.matrix = as.dist(1 - connect.matrix); HC = hclust(dist.matrix, "average");
//   rho = cor(dist.matrix, cophenetic(HC)); membership = cutree(HC, k); HC$order.
// Restated from the published algorithms R's stats package uses (R itself is absent from the image,
// so parity with R is unpinned; tests cross-check against scipy's average linkage):
//   * F. Murtagh's nearest-neighbour-list agglomeration with Lance-Williams group-average update
//     (R's hclust.f, including the nearest-neighbour fix for i2 > k),
//   * the merge/order post-processing of R's hcass2,
//   * cophenetic heights from the merge sequence, Pearson correlation with long-double sums.
// n <= a few thousand (consensus matrices are n x n), so O(n^2) memory and time are fine here.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

#include "../../include/nmfc.h"

namespace {

// packed index of pair (i < j), 0-based, row-wise upper triangle
inline long ioffst(long n, long i, long j) { return j + i * n - (i + 1) * (i + 2) / 2; }

// First index t of the minimum of d[0..len) if that minimum is strictly below `best` (which it then becomes), else -1:
// the scan `if (d[t] < best) { best = d[t]; at = t; }` of R's hclust.f, in two passes (a four-way min, then the first
// index holding it) so the compiler can keep four independent chains instead of one.
int first_min(const double* d, int len, double& best) {
  double m0 = best, m1 = best, m2 = best, m3 = best;
  int t = 0;
  for (; t + 4 <= len; t += 4) {
    m0 = d[t] < m0 ? d[t] : m0;
    m1 = d[t + 1] < m1 ? d[t + 1] : m1;
    m2 = d[t + 2] < m2 ? d[t + 2] : m2;
    m3 = d[t + 3] < m3 ? d[t + 3] : m3;
  }
  for (; t < len; ++t) m0 = d[t] < m0 ? d[t] : m0;
  const double m01 = m1 < m0 ? m1 : m0, m23 = m3 < m2 ? m3 : m2, m = m23 < m01 ? m23 : m01;
  if (!(m < best)) return -1;
  best = m;
  for (t = 0; t < len; ++t)
    if (d[t] == m) return t;
  return -1;
}

void hclust_average(int n, std::vector<double>& diss, std::vector<int>& ia, std::vector<int>& ib,
                    std::vector<double>& crit) {
  const double INF = 1e300;
  std::vector<char> flag(n, 1);
  std::vector<int> nn(n, 0);
  std::vector<double> disnn(n, INF), membr(n, 1.0);
  ia.assign(n, 0);
  ib.assign(n, 0);
  crit.assign(n, 0.0);
  int im = 0, jj = 0, jm = 0;
  // row i's pairs (i, j > i) are contiguous in the packed triangle
  for (int i = 0; i < n - 1; ++i) {
    double dmin = INF;
    const int t = first_min(&diss[ioffst(n, i, i + 1)], n - 1 - i, dmin);
    if (t >= 0) jm = i + 1 + t;
    nn[i] = jm;
    disnn[i] = dmin;
  }
  int ncl = n;
  while (ncl > 1) {
    double dmin = INF;
    for (int i = 0; i < n - 1; ++i) {
      if (flag[i] && disnn[i] < dmin) {
        dmin = disnn[i];
        im = i;
        jm = nn[i];
      }
    }
    --ncl;
    const int i2 = im < jm ? im : jm;
    const int j2 = im < jm ? jm : im;
    ia[n - ncl - 1] = i2;
    ib[n - ncl - 1] = j2;
    crit[n - ncl - 1] = dmin;
    flag[j2] = 0;
    dmin = INF;
    for (int k = 0; k < n; ++k) {
      if (flag[k] && k != i2) {
        const long ind1 = (i2 < k) ? ioffst(n, i2, k) : ioffst(n, k, i2);
        const long ind2 = (j2 < k) ? ioffst(n, j2, k) : ioffst(n, k, j2);
        diss[ind1] = (membr[i2] * diss[ind1] + membr[j2] * diss[ind2]) / (membr[i2] + membr[j2]);
        if (i2 < k) {
          if (diss[ind1] < dmin) {
            dmin = diss[ind1];
            jj = k;
          }
        } else {
          if (diss[ind1] < disnn[k]) {
            disnn[k] = diss[ind1];
            nn[k] = i2;
          }
        }
      }
    }
    membr[i2] += membr[j2];
    disnn[i2] = dmin;
    nn[i2] = jj;
    // cluster j2 is gone: its pairs read INF from now on, so the rescans below need no liveness test (an INF never
    // beats the INF they start from, as a dead j never entered R's scan)
    for (int k = 0; k < j2; ++k) diss[ioffst(n, k, j2)] = INF;
    for (int k = j2 + 1; k < n; ++k) diss[ioffst(n, j2, k)] = INF;
    for (int i = 0; i < n - 1; ++i) {
      if (flag[i] && (nn[i] == i2 || nn[i] == j2)) {
        double dm = INF;
        const int t = first_min(&diss[ioffst(n, i, i + 1)], n - 1 - i, dm);
        if (t >= 0) jj = i + 1 + t;
        nn[i] = jj;
        disnn[i] = dm;
      }
    }
  }
}

// R's hcass2: merge matrix in R's convention (negative = singleton, positive = earlier merge, both
// 1-based) and the leaf order.
void hcass2(int n, const std::vector<int>& ia0, const std::vector<int>& ib0, std::vector<int>& iia,
            std::vector<int>& iib, std::vector<int>& iorder) {
  std::vector<int> ia(n), ib(n);
  for (int i = 0; i < n; ++i) {
    ia[i] = ia0[i] + 1;
    ib[i] = ib0[i] + 1;
  }
  iia = ia;
  iib = ib;
  for (int i = 0; i < n - 2; ++i) {
    const int k = ia[i] < ib[i] ? ia[i] : ib[i];
    for (int j = i + 1; j < n - 1; ++j) {
      if (ia[j] == k) iia[j] = -(i + 1);
      if (ib[j] == k) iib[j] = -(i + 1);
    }
  }
  for (int i = 0; i < n - 1; ++i) {
    iia[i] = -iia[i];
    iib[i] = -iib[i];
  }
  for (int i = 0; i < n - 1; ++i) {
    if (iia[i] > 0 && iib[i] < 0) {
      const int k = iia[i];
      iia[i] = iib[i];
      iib[i] = k;
    }
    if (iia[i] > 0 && iib[i] > 0) {
      const int k1 = iia[i] < iib[i] ? iia[i] : iib[i];
      const int k2 = iia[i] < iib[i] ? iib[i] : iia[i];
      iia[i] = k1;
      iib[i] = k2;
    }
  }
  iorder.assign(n + 1, 0);
  iorder[0] = iia[n - 2];
  iorder[1] = iib[n - 2];
  int loc = 2;
  for (int i = n - 2; i >= 1; --i) {
    for (int j = 0; j < loc; ++j) {
      if (iorder[j] == i) {
        iorder[j] = iia[i - 1];
        if (j == loc - 1) {
          ++loc;
          iorder[loc - 1] = iib[i - 1];
        } else {
          ++loc;
          for (int k = loc - 1; k >= j + 2; --k) iorder[k] = iorder[k - 1];
          iorder[j + 1] = iib[i - 1];
        }
        break;
      }
    }
  }
  for (int i = 0; i < n; ++i) iorder[i] = -iorder[i];
  iorder.resize(n);
}

}  // namespace

extern "C" {

double nmfc_cophenetic(const double* C, int n, int32_t* order_out, int32_t* merge_out, double* height_out) {
  if (n < 2) return NAN;
  const long npair = (long)n * (n - 1) / 2;
  std::vector<double> d0(npair);
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) d0[ioffst(n, i, j)] = 1.0 - C[(long)j * n + i];   // as.dist takes the lower triangle
  // as.dist(1 - C) reads C[j, i] for i < j (column-major lower triangle); C is symmetric here
  std::vector<double> diss = d0;
  std::vector<int> ia, ib, iia, iib, iorder;
  std::vector<double> crit;
  hclust_average(n, diss, ia, ib, crit);
  hcass2(n, ia, ib, iia, iib, iorder);
  if (order_out)
    for (int i = 0; i < n; ++i) order_out[i] = iorder[i];
  if (merge_out)
    for (int i = 0; i < n - 1; ++i) {
      merge_out[2 * i] = iia[i];
      merge_out[2 * i + 1] = iib[i];
    }
  if (height_out)
    for (int i = 0; i < n - 1; ++i) height_out[i] = crit[i];
  // cophenetic distances from the merge sequence
  std::vector<std::vector<int>> members(n - 1);
  std::vector<double> coph(npair, 0.0);
  auto mem_of = [&](int code, std::vector<int>& out) {
    if (code < 0)
      out.push_back(-code - 1);
    else
      out.insert(out.end(), members[code - 1].begin(), members[code - 1].end());
  };
  for (int s = 0; s < n - 1; ++s) {
    std::vector<int> a, b;
    mem_of(iia[s], a);
    mem_of(iib[s], b);
    for (int x : a)
      for (int y : b) coph[x < y ? ioffst(n, x, y) : ioffst(n, y, x)] = crit[s];
    members[s] = a;
    members[s].insert(members[s].end(), b.begin(), b.end());
    if (iia[s] > 0) std::vector<int>().swap(members[iia[s] - 1]);
    if (iib[s] > 0) std::vector<int>().swap(members[iib[s] - 1]);
  }
  // Pearson correlation over the pairs, R-style: means with a correction pass, long-double sums
  long double sx = 0, sy = 0;
  for (long q = 0; q < npair; ++q) {
    sx += d0[q];
    sy += coph[q];
  }
  long double mx = sx / npair, my = sy / npair, cx = 0, cy = 0;
  for (long q = 0; q < npair; ++q) {
    cx += d0[q] - mx;
    cy += coph[q] - my;
  }
  mx += cx / npair;
  my += cy / npair;
  long double sxy = 0, sxx = 0, syy = 0;
  for (long q = 0; q < npair; ++q) {
    const long double dx = d0[q] - mx, dy = coph[q] - my;
    sxy += dx * dy;
    sxx += dx * dx;
    syy += dy * dy;
  }
  if (sxx <= 0 || syy <= 0) return NAN;
  return (double)(sxy / (sqrtl(sxx) * sqrtl(syy)));
}

int nmfc_cophenetic_batch(const double* C, int nk, int n, int nthreads, double* rho_out, int32_t* order_out,
                          int32_t* merge_out, double* height_out) {
  if (!C || nk < 1 || n < 2 || !rho_out) return -1;
  if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
  nthreads = std::min(nthreads, nk);
  const long nn = (long)n * n;
  std::atomic<int> next(0);
  auto work = [&] {
    for (int q; (q = next.fetch_add(1)) < nk;)
      rho_out[q] = nmfc_cophenetic(C + q * nn, n, order_out ? order_out + (long)q * n : nullptr,
                                   merge_out ? merge_out + (long)q * 2 * (n - 1) : nullptr,
                                   height_out ? height_out + (long)q * (n - 1) : nullptr);
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nthreads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  return 0;
}

int nmfc_cutree(const int32_t* merge, int n, int k, int32_t* membership_out) {
  if (n < 1 || k < 1 || k > n) return -1;
  std::vector<int> parent(n);
  for (int i = 0; i < n; ++i) parent[i] = i;
  auto find = [&](int x) {
    while (parent[x] != x) x = parent[x] = parent[parent[x]];
    return x;
  };
  std::vector<int> rep(n - 1 > 0 ? n - 1 : 1, 0);   // a representative observation of each merge
  for (int s = 0; s < n - k; ++s) {
    const int a = merge[2 * s], b = merge[2 * s + 1];
    const int ra = a < 0 ? -a - 1 : rep[a - 1];
    const int rb = b < 0 ? -b - 1 : rep[b - 1];
    const int fa = find(ra), fb = find(rb);
    parent[fb] = fa;
    rep[s] = fa;
  }
  // clusters numbered by order of first appearance over the observations
  std::vector<int> id(n, 0);
  int next = 0;
  for (int i = 0; i < n; ++i) {
    const int r = find(i);
    if (!id[r]) id[r] = ++next;
    membership_out[i] = id[r];
  }
  return 0;
}

}  // extern "C"
