"""TEST INFRASTRUCTURE ONLY: a line-by-line Python restatement of what R's stats package runs for
nmf.r:166-177 (`HC = hclust(as.dist(1 - C), method = "average")`, `HC$order`, `cutree(HC, k)`), used
to check nmfconsensus_amd's host C++ (nmfconsensus_amd/csrc/hclust.cpp) on tied and untied inputs.

Restated from the published R sources (R is absent from this image, so this checker is itself unpinned
against a running R; it fixes the tie rules those sources define):
  * hclust.f  HCLUST: F. Murtagh's nearest-neighbour-list agglomeration, Lance-Williams group-average
    update, with R's nearest-neighbour fix for k < i2.  Tie rules: the first NN list keeps the FIRST j
    with the minimum (`IF (DMIN .GT. DISS(IND))`); the pair to merge is the FIRST i in 1..n-1 with the
    smallest DISNN (`DISNN(I) .LT. DMIN`); row rescans keep the first j (`.LT.`).
  * hclust.f  HCASS2: merge matrix in S/R convention and the leaf order.
  * hclust-utils.c  cutree: after merge step n - k, clusters numbered in order of first appearance of
    the observations 1..n.
All indices here are 1-based like the Fortran.
"""
from __future__ import annotations

import numpy as np

INF = 1.0e300


def ioffst(n, i, j):
    """1-based packed index of pair (i < j) in a dist vector (hclust.f IOFFST)."""
    return j + (i - 1) * n - (i * (i + 1)) // 2


def dist_from_consensus(C):
    """as.dist(1 - C): the lower triangle, column-major -> diss[ioffst(i, j)] = (1 - C)[j, i]."""
    C = np.asarray(C, dtype=np.float64)
    n = C.shape[0]
    diss = [0.0] * (n * (n - 1) // 2 + 1)   # 1-based
    for i in range(1, n):
        for j in range(i + 1, n + 1):
            diss[ioffst(n, i, j)] = 1.0 - C[j - 1, i - 1]
    return diss


def hclust_average(n, diss):
    """HCLUST with IOPT = 3 (group average).  Returns ia, ib, crit (1-based lists, length n+1)."""
    diss = list(diss)
    ia = [0] * (n + 1)
    ib = [0] * (n + 1)
    crit = [0.0] * (n + 1)
    membr = [1.0] * (n + 1)
    nn = [0] * (n + 1)
    disnn = [0.0] * (n + 1)
    flag = [True] * (n + 1)
    ncl = n
    im = jj = jm = 0
    for i in range(1, n):
        dmin = INF
        for j in range(i + 1, n + 1):
            ind = ioffst(n, i, j)
            if dmin > diss[ind]:
                dmin = diss[ind]
                jm = j
        nn[i] = jm
        disnn[i] = dmin
    while ncl > 1:
        dmin = INF
        for i in range(1, n):
            if flag[i] and disnn[i] < dmin:
                dmin = disnn[i]
                im = i
                jm = nn[i]
        ncl -= 1
        i2, j2 = min(im, jm), max(im, jm)
        ia[n - ncl] = i2
        ib[n - ncl] = j2
        crit[n - ncl] = dmin
        flag[j2] = False
        dmin = INF
        for k in range(1, n + 1):
            if flag[k] and k != i2:
                ind1 = ioffst(n, i2, k) if i2 < k else ioffst(n, k, i2)
                ind2 = ioffst(n, j2, k) if j2 < k else ioffst(n, k, j2)
                diss[ind1] = (membr[i2] * diss[ind1] + membr[j2] * diss[ind2]) / (membr[i2] + membr[j2])
                if i2 < k:
                    if diss[ind1] < dmin:
                        dmin = diss[ind1]
                        jj = k
                else:
                    if diss[ind1] < disnn[k]:
                        disnn[k] = diss[ind1]
                        nn[k] = i2
        membr[i2] += membr[j2]
        disnn[i2] = dmin
        nn[i2] = jj
        for i in range(1, n):
            if flag[i] and (nn[i] == i2 or nn[i] == j2):
                dmin = INF
                for j in range(i + 1, n + 1):
                    if flag[j]:
                        ind = ioffst(n, i, j)
                        if diss[ind] < dmin:
                            dmin = diss[ind]
                            jj = j
                nn[i] = jj
                disnn[i] = dmin
    return ia, ib, crit


def hcass2(n, ia, ib):
    """HCASS2: returns iia, iib (merge matrix columns) and iorder (all 1-based lists, length n+1)."""
    iia = list(ia)
    iib = list(ib)
    for i in range(1, n - 1):
        k = min(ia[i], ib[i])
        for j in range(i + 1, n):
            if ia[j] == k:
                iia[j] = -i
            if ib[j] == k:
                iib[j] = -i
    for i in range(1, n):
        iia[i] = -iia[i]
        iib[i] = -iib[i]
    for i in range(1, n):
        if iia[i] > 0 and iib[i] < 0:
            iia[i], iib[i] = iib[i], iia[i]
        if iia[i] > 0 and iib[i] > 0:
            k1, k2 = min(iia[i], iib[i]), max(iia[i], iib[i])
            iia[i], iib[i] = k1, k2
    iorder = [0] * (n + 2)
    iorder[1] = iia[n - 1]
    iorder[2] = iib[n - 1]
    loc = 2
    for i in range(n - 2, 0, -1):
        for j in range(1, loc + 1):
            if iorder[j] == i:
                iorder[j] = iia[i]
                if j == loc:
                    loc += 1
                    iorder[loc] = iib[i]
                else:
                    loc += 1
                    for k in range(loc, j + 1, -1):
                        iorder[k] = iorder[k - 1]
                    iorder[j + 1] = iib[i]
                break
    for i in range(1, n + 1):
        iorder[i] = -iorder[i]
    return iia, iib, iorder


def cutree(n, merge, k):
    """hclust-utils.c cutree for one k: merge is (n-1) x 2 (R convention); returns memberships 1..n."""
    if k == n:
        return list(range(1, n + 1))
    sing = [True] * (n + 1)
    m_nr = [0] * (n + 1)
    ans = None
    for step in range(1, n):
        m1, m2 = int(merge[step - 1][0]), int(merge[step - 1][1])
        if m1 < 0 and m2 < 0:
            m_nr[-m1] = m_nr[-m2] = step
            sing[-m1] = sing[-m2] = False
        elif m1 < 0 or m2 < 0:
            if m1 < 0:
                j, m1 = -m1, m2
            else:
                j = -m2
            for l in range(1, n + 1):
                if m_nr[l] == m1:
                    m_nr[l] = step
            m_nr[j] = step
            sing[j] = False
        else:
            for l in range(1, n + 1):
                if m_nr[l] == m1 or m_nr[l] == m2:
                    m_nr[l] = step
        if k == n - step:
            z = [0] * (n + 1)
            nclust = 0
            ans = [0] * n
            for l in range(1, n + 1):
                if sing[l]:
                    nclust += 1
                    ans[l - 1] = nclust
                else:
                    if z[m_nr[l]] == 0:
                        nclust += 1
                        z[m_nr[l]] = nclust
                    ans[l - 1] = z[m_nr[l]]
    return ans


def r_hclust_consensus(C):
    """(order, merge, height) of hclust(as.dist(1 - C), "average") as R computes them."""
    n = np.asarray(C).shape[0]
    ia, ib, crit = hclust_average(n, dist_from_consensus(C))
    iia, iib, iorder = hcass2(n, ia, ib)
    merge = np.array([[iia[i], iib[i]] for i in range(1, n)], dtype=np.int32)
    return np.array(iorder[1:n + 1], dtype=np.int32), merge, np.array(crit[1:n], dtype=np.float64)
