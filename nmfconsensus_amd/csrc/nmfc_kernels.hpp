// nmfc_kernels.hpp -- HIP kernels of the batched MU restart engine (gfx950 / CDNA4).
//
// Device layouts (DESIGN.md "Data layout in HBM"):
//   Acm [n_cols_pad][m_pad]  column j of A, K(=gene)-contiguous        (operand of W^T A)
//   Arm [m_pad][n_pad]       row i of A, K(=sample)-contiguous          (operand of A H^T)
//   W   [Kt_pad][m_pad]      column c of the stacked W_all (restart r owns columns col0..col0+k-1)
//   H   [Kt_pad][n_pad]      row c of the stacked H_all (row-major, sample-contiguous)
//   restarts are packed into panels of 64 columns; a restart never straddles a panel.
// Both big contractions are "TN" tiles: C[r][c] = sum_k P[r][k] * Q[c][k] with K-contiguous rows,
// computed with v_mfma_f64_16x16x4_f64 from LDS-staged 64x32 tiles.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nmfc {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

constexpr int TILE = 64;           // output tile edge == panel width (restart columns)
constexpr int BK = 32;             // K depth of one LDS stage
constexpr int LDSS = BK + 2;       // LDS row stride (doubles): 272 B rows -> conflict-free b64 fragment reads
constexpr int NT = 256;            // threads per workgroup (4 waves, 2x2 over the 64x64 tile)
constexpr int HCH = 256;           // sample chunk of the H-update kernel
constexpr int KMAX = 16;           // largest rank k handled by the H-update LDS arrays
constexpr int STOP_FIXED = 0, STOP_REF_COMPAT = 1, STOP_ARGMAX_STABLE = 2;
constexpr double DIV_BY_ZERO_AVOIDANCE = 1E-09;   // nmf_mu.c:56

// nmf_mu.c:184-191 / :209-216: h = (h0 == 0 || num == 0) ? 0 : h0 * (num / (den + 1e-9)); clamp < 0
// (ZERO_THRESHOLD = 0.0, common.h:15).  Order add -> divide -> multiply is kept (no contraction).
__device__ __forceinline__ double mu_rule(double old, double num, double den) {
  if (old == 0.0 || num == 0.0) return 0.0;
  const double q = num / (den + DIV_BY_ZERO_AVOIDANCE);
  const double t = old * q;
  return t < 0.0 ? 0.0 : t;
}

// One 64x64 fp64 output tile, K range [kbeg, kend) (multiple of BK), 256 threads.
// acc[mb][nb] holds the 16x16 block (wr*32+mb*16, wc*32+nb*16) of the wave's 32x32 quadrant.
// C/D map of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 * reg.
__device__ __forceinline__ void tile_tn_f64(const double* __restrict__ P, long ldp, const double* __restrict__ Q,
                                            long ldq, int kbeg, int kend, double* __restrict__ smem,
                                            d4 (&acc)[2][2]) {
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63;
  const int wr = w >> 1, wc = w & 1;
  double* Ps = smem;
  double* Qs = smem + 2 * TILE * LDSS;
  const int lrow = w * 16 + (l >> 4);
  const int lch = (l & 15) * 2;
  d2 pr[4], qr[4];
  const int nst = (kend - kbeg) / BK;

#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = lrow + 4 * i;
    pr[i] = *reinterpret_cast<const d2*>(P + (long)row * ldp + kbeg + lch);
    qr[i] = *reinterpret_cast<const d2*>(Q + (long)row * ldq + kbeg + lch);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = lrow + 4 * i;
    *reinterpret_cast<d2*>(Ps + row * LDSS + lch) = pr[i];
    *reinterpret_cast<d2*>(Qs + row * LDSS + lch) = qr[i];
  }
  __syncthreads();

  const int fr = l & 15, fk = l >> 4;
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    if (s + 1 < nst) {
      const int k0 = kbeg + (s + 1) * BK;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = lrow + 4 * i;
        pr[i] = *reinterpret_cast<const d2*>(P + (long)row * ldp + k0 + lch);
        qr[i] = *reinterpret_cast<const d2*>(Q + (long)row * ldq + k0 + lch);
      }
    }
    const double* Pb = Ps + buf * TILE * LDSS;
    const double* Qb = Qs + buf * TILE * LDSS;
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      const int kc = kk * 4 + fk;
      const double a0 = Pb[(wr * 32 + fr) * LDSS + kc];
      const double a1 = Pb[(wr * 32 + 16 + fr) * LDSS + kc];
      const double b0 = Qb[(wc * 32 + fr) * LDSS + kc];
      const double b1 = Qb[(wc * 32 + 16 + fr) * LDSS + kc];
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (s + 1 < nst) {
      double* Pn = Ps + (buf ^ 1) * TILE * LDSS;
      double* Qn = Qs + (buf ^ 1) * TILE * LDSS;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = lrow + 4 * i;
        *reinterpret_cast<d2*>(Pn + row * LDSS + lch) = pr[i];
        *reinterpret_cast<d2*>(Qn + row * LDSS + lch) = qr[i];
      }
    }
    __syncthreads();
  }
}

__device__ __forceinline__ int acc_row(int wr, int mb, int l, int reg) { return wr * 32 + mb * 16 + (l >> 4) + 4 * reg; }
__device__ __forceinline__ int acc_col(int wc, int nb, int l) { return wc * 32 + nb * 16 + (l & 15); }

// A panel takes part in an iteration when one of its restarts is still running, or (for the
// W update) stopped at exactly this iteration.
__device__ __forceinline__ bool panel_live(const int* __restrict__ prb, const int* __restrict__ pre, int p,
                                           const int* __restrict__ stop_iter, int iter) {
  const int b = prb[p], e = pre[p];
  for (int r = b; r < e; ++r) {
    const int s = stop_iter[r];
    if (s == 0 || s == iter) return true;
  }
  return false;
}

// ---------------------------------------------------------------------------------------------
// K1 "wta":  G = W^T A  (nmf_mu.c:174) and SW = W_p^T W_p (nmf_mu.c:176) for every live panel.
// grid = nsplit x npanels x (ntj + 1); column tile t == ntj is the panel Gram tile.  The gene
// range is cut into fixed chunks (a function of m only), so the reduction order of every entry is
// independent of batch composition; partials are summed in chunk order by K2.
// ---------------------------------------------------------------------------------------------
static __global__ __launch_bounds__(NT) void k_wta(const double* __restrict__ W, const double* __restrict__ Acm, long m_pad,
                                            int npanels, int ntj, int kchunk, const int* __restrict__ prb,
                                            const int* __restrict__ pre, const int* __restrict__ stop_iter, int iter,
                                            double* __restrict__ Gpart, long g_ld, long g_split,
                                            double* __restrict__ SWpart, long sw_split) {
  __shared__ __attribute__((aligned(16))) double smem[4 * TILE * LDSS];
  const int ntiles = ntj + 1;
  const int b = blockIdx.x;
  const int t = b % ntiles;
  const int rest = b / ntiles;
  const int p = rest % npanels;
  const int s = rest / npanels;
  if (!panel_live(prb, pre, p, stop_iter, 0x7fffffff) ) return;   // only still-running restarts
  const double* P = W + (long)p * TILE * m_pad;
  const bool gram = (t == ntj);
  const double* Q = gram ? P : Acm + (long)t * TILE * m_pad;
  const int kbeg = s * kchunk;
  const int kend = min((long)kbeg + kchunk, m_pad);
  d4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
  tile_tn_f64(P, m_pad, Q, m_pad, kbeg, kend, smem, acc);
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  double* out;
  long ld;
  if (gram) {
    out = SWpart + (long)s * sw_split + (long)p * TILE * TILE;
    ld = TILE;
  } else {
    out = Gpart + (long)s * g_split + (long)p * TILE * g_ld + (long)t * TILE;
    ld = g_ld;
  }
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) out[(long)acc_row(wr, mb, l, reg) * ld + acc_col(wc, nb, l)] = acc[mb][nb][reg];
  (void)iter;
}

// ---------------------------------------------------------------------------------------------
// K2 "hupdate": one workgroup per running restart.
//   work2 = SW * H (nmf_mu.c:178); H <- mu_rule(H, G, work2) (:184-191); SH = H H^T (:200);
//   stability check on the new H at even iterations (:253-282).
// ---------------------------------------------------------------------------------------------
struct RestartInfo {
  int col0;   // first global column of the restart in W / H
  int k;
};

static __global__ __launch_bounds__(NT) void k_hupdate(int iter, int maxiter, int stop_rule, const RestartInfo* __restrict__ ri,
                                                int n, long n_pad, const double* __restrict__ Gpart, long g_ld,
                                                long g_split, int nsplit, const double* __restrict__ SWpart,
                                                long sw_split, double* __restrict__ H, double* __restrict__ SHp,
                                                int* __restrict__ stop_iter, int* __restrict__ stop_reason,
                                                int* __restrict__ unchanged, int* __restrict__ classes, long cls_ld,
                                                int* __restrict__ n_stopped) {
  __shared__ double sw[KMAX * KMAX];
  __shared__ double Hc[KMAX * HCH];
  __shared__ double Hn[KMAX * HCH];
  __shared__ double win[KMAX * KMAX];
  __shared__ int changed;
  const int r = blockIdx.x;
  if (stop_iter[r] != 0) return;
  const int tid = threadIdx.x;
  const int c0 = ri[r].col0, k = ri[r].k;
  const int p = c0 / TILE, lc0 = c0 % TILE;
  const bool check = (stop_rule != STOP_FIXED) && iter > 1 && (iter % 2 == 0);
  if (tid == 0) changed = 0;
  for (int idx = tid; idx < k * k; idx += NT) {
    const int a = idx / k, bb = idx % k;
    const long off = (long)p * TILE * TILE + (long)(lc0 + a) * TILE + (lc0 + bb);
    double sacc = SWpart[off];
    for (int sp = 1; sp < nsplit; ++sp) sacc += SWpart[(long)sp * sw_split + off];
    sw[a * KMAX + bb] = sacc;
  }
  for (int idx = tid; idx < KMAX * KMAX; idx += NT) win[idx] = 0.0;
  const int npairs = k * (k + 1) / 2;
  int pa = 0, pb = 0;
  if (tid < npairs) {  // (pa, pb) = tid-th pair of the upper triangle, row-major
    int t = tid;
    while (t >= k - pa) { t -= k - pa; ++pa; }
    pb = pa + t;
  }
  double shacc = 0.0;
  __syncthreads();

  for (int j0 = 0; j0 < n; j0 += HCH) {
    const int j = j0 + tid;
    const bool valid = j < n;
    for (int a = 0; a < k; ++a) Hc[a * HCH + tid] = valid ? H[(long)(c0 + a) * n_pad + j] : 0.0;
    int best = 0;
    for (int a = 0; a < k; ++a) {
      double hn = 0.0;
      if (valid) {
        const long goff = (long)(c0 + a) * g_ld + j;
        double g = Gpart[goff];
        for (int sp = 1; sp < nsplit; ++sp) g += Gpart[(long)sp * g_split + goff];
        double d = 0.0;
        for (int bb = 0; bb < k; ++bb) d = fma(sw[a * KMAX + bb], Hc[bb * HCH + tid], d);
        hn = mu_rule(Hc[a * HCH + tid], g, d);
        H[(long)(c0 + a) * n_pad + j] = hn;
        if (stop_rule == STOP_REF_COMPAT) {
          // flat column-major index of (a, j) in the k x n buffer; window i reads [i*n, i*n+k)
          const long tf = (long)j * k + a;
          const long wi = tf / n;
          if (wi < k) {
            const long wj = tf - wi * n;
            if (wj < k) win[wi * KMAX + wj] = hn;
          }
        }
      }
      Hn[a * HCH + tid] = hn;
      if (a > 0 && hn > Hn[best * HCH + tid]) best = a;
    }
    if (check && stop_rule == STOP_ARGMAX_STABLE && valid) {
      int* cl = classes + (long)r * cls_ld + j;
      if (*cl != best) {
        *cl = best;
        changed = 1;
      }
    }
    __syncthreads();
    if (tid < npairs) {
      const int cnt = min(HCH, n - j0);
      const double* ha = Hn + pa * HCH;
      const double* hb = Hn + pb * HCH;
      for (int q = 0; q < cnt; ++q) shacc = fma(ha[q], hb[q], shacc);
    }
    __syncthreads();
  }
  if (tid < npairs) {
    double* sh = SHp + (long)p * TILE * TILE;
    sh[(lc0 + pa) * TILE + (lc0 + pb)] = shacc;
    sh[(lc0 + pb) * TILE + (lc0 + pa)] = shacc;
  }
  if (check && stop_rule == STOP_REF_COMPAT) {
    const int nwin = k < n ? k : n;
    if (tid < nwin) {
      int c = 0;
      for (int jj = 1; jj < k; ++jj)
        if (win[tid * KMAX + jj] > win[tid * KMAX + jj - 1]) c = jj;
      int* cl = classes + (long)r * cls_ld + tid;
      if (*cl != c) {
        *cl = c;
        changed = 1;
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    int reason = 0;
    if (check) {
      if (!changed) {
        const int u = unchanged[r] + 1;
        unchanged[r] = u;
        if (u >= 200) reason = 1;   // nmf_mu.c:269-271
      } else {
        unchanged[r] = 0;
      }
    }
    if (!reason && iter >= maxiter) reason = 2;
    if (reason) {
      stop_iter[r] = iter;
      stop_reason[r] = reason;
      atomicAdd(n_stopped, 1);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// K3 "ahtw": F = A h^T (nmf_mu.c:198) computed transposed per tile (rows = panel columns c, cols =
// genes i), fused with work2w = W0 * (h h^T) (:202) and the W rule (:209-216), written in place.
// grid = npanels x ngt (gene tiles fastest).
// ---------------------------------------------------------------------------------------------
static __global__ __launch_bounds__(NT) void k_ahtw(int iter, const double* __restrict__ H, long n_pad,
                                             const double* __restrict__ Arm, long m_pad, double* __restrict__ W,
                                             const double* __restrict__ SHp, const int* __restrict__ pcol_start,
                                             const int* __restrict__ pcol_k, const int* __restrict__ pcol_rest,
                                             const int* __restrict__ prb, const int* __restrict__ pre,
                                             const int* __restrict__ stop_iter, int ngt) {
  __shared__ __attribute__((aligned(16))) double smem[4 * TILE * LDSS];
  __shared__ int cs[TILE], ck[TILE], cact[TILE];
  const int b = blockIdx.x;
  const int g = b % ngt;
  const int p = b / ngt;
  if (!panel_live(prb, pre, p, stop_iter, iter)) return;
  const double* P = H + (long)p * TILE * n_pad;
  const double* Q = Arm + (long)g * TILE * n_pad;
  d4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
  tile_tn_f64(P, n_pad, Q, n_pad, 0, (int)n_pad, smem, acc);

  // epilogue: W tile (64 panel columns x 64 genes) and the panel's h h^T blocks into LDS
  constexpr int ES = TILE + 1;
  double* Wl = smem;
  double* Sl = smem + TILE * ES;
  const int tid = threadIdx.x;
  for (int idx = tid; idx < TILE * TILE; idx += NT) {
    const int c = idx / TILE, i = idx % TILE;
    Wl[c * ES + i] = W[((long)p * TILE + c) * m_pad + (long)g * TILE + i];
    Sl[c * ES + i] = SHp[(long)p * TILE * TILE + idx];
  }
  if (tid < TILE) {
    const int pc = p * TILE + tid;
    cs[tid] = pcol_start[pc];
    ck[tid] = pcol_k[pc];
    const int rr = pcol_rest[pc];
    int act = 0;
    if (rr >= 0) {
      const int s = stop_iter[rr];
      act = (s == 0 || s == iter);
    }
    cact[tid] = act;
  }
  __syncthreads();
  const int l = tid & 63, w = tid >> 6, wr = w >> 1, wc = w & 1;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int c = acc_row(wr, mb, l, reg);
        const int i = acc_col(wc, nb, l);
        if (!cact[c]) continue;
        const int st = cs[c], kk = ck[c];
        double e = 0.0;
        for (int q = 0; q < kk; ++q) e = fma(Sl[c * ES + st + q], Wl[(st + q) * ES + i], e);
        const double wn = mu_rule(Wl[c * ES + i], acc[mb][nb][reg], e);
        W[((long)p * TILE + c) * m_pad + (long)g * TILE + i] = wn;
      }
}

// ---------------------------------------------------------------------------------------------
// Init: generateMatrix(ran) (generatematrix.c:131-137) with randnumber (randnumber.c:34) over the
// glibc TYPE_3 stream seeded per job.  Thread = (restart, chunk of CHUNK draws).  The chunk's start
// state is J[c] * s_344 (mod 2^32), J[c] = M^(c*CHUNK) the 31x31 jump matrix of the lagged
// recurrence r[i] = r[i-31] + r[i-3].
// ---------------------------------------------------------------------------------------------
constexpr int RCHUNK = 31 * 32;   // draws per thread (multiple of 31 for a statically indexed ring)

struct InitJob {
  uint32_t seed;
  int col0;
  int k;
  int nchunks;
};

static __global__ __launch_bounds__(NT) void k_init(const InitJob* __restrict__ jobs, const int* __restrict__ chunk_job,
                                             const int* __restrict__ chunk_idx, int total_chunks,
                                             const uint32_t* __restrict__ jump, int m, int n, long m_pad, long n_pad,
                                             int min_init, int max_init, double* __restrict__ W,
                                             double* __restrict__ H) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total_chunks) return;
  const InitJob jb = jobs[chunk_job[gid]];
  const int c = chunk_idx[gid];
  // srand(seed): r[0..30] by the Park-Miller LCG (Schrage), r[31..33] = r[0..2]
  uint32_t ring[31];
  int32_t word = (int32_t)(jb.seed ? jb.seed : 1u);
  ring[0] = (uint32_t)word;
#pragma unroll
  for (int i = 1; i < 31; ++i) {
    long hi = word / 127773;
    long lo = word % 127773;
    long wv = 16807 * lo - 2836 * hi;
    if (wv < 0) wv += 2147483647;
    word = (int32_t)wv;
    ring[i] = (uint32_t)word;
  }
  // ring[q] holds r[q]; r[31..33] = r[0..2] occupy the same slots.  Steps i = 34..343 (10 x 31).
#pragma unroll 1
  for (int blk = 0; blk < 10; ++blk) {
#pragma unroll
    for (int q = 0; q < 31; ++q) {
      const int pos = (3 + q) % 31;
      ring[pos] = ring[pos] + ring[(pos + 28) % 31];
    }
  }
  // ordered window s[q] = r[313 + q] sits at ring[(3 + q) % 31]
  uint32_t s[31];
#pragma unroll
  for (int q = 0; q < 31; ++q) s[q] = ring[(3 + q) % 31];
  if (c > 0) {
    const uint32_t* J = jump + (long)c * 31 * 31;
#pragma unroll
    for (int q = 0; q < 31; ++q) {
      uint32_t v = 0;
#pragma unroll
      for (int pq = 0; pq < 31; ++pq) v += J[q * 31 + pq] * s[pq];
      ring[q] = v;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 31; ++q) ring[q] = s[q];
  }
  // ring[q] = r[i0 - 31 + q]; step jj overwrites slot jj % 31 with r[i0+jj] = slot + slot[(jj+28)%31]
  const long mk = (long)m * jb.k;
  const long total = mk + (long)jb.k * n;
  long t = (long)c * RCHUNK;
#pragma unroll 1
  for (int blk = 0; blk < RCHUNK / 31; ++blk) {
#pragma unroll
    for (int q = 0; q < 31; ++q) {
      const uint32_t v = ring[q] + ring[(q + 28) % 31];
      ring[q] = v;
      if (t < total) {
        const int32_t o = (int32_t)(v >> 1);
        const int32_t prod = (int32_t)((uint32_t)(max_init - min_init) * (uint32_t)o);
        const double val = (double)min_init + (double)prod / 2147483647.0;
        if (t < mk) {
          const long a = t / m, i = t - a * m;
          W[(long)(jb.col0 + a) * m_pad + i] = val;
        } else {
          const long tt = t - mk;
          const long jcol = tt / jb.k, a = tt - jcol * jb.k;
          H[(long)(jb.col0 + a) * n_pad + jcol] = val;
        }
      }
      ++t;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Labels (nmf.r:128 / documented intent) and connectivity counts (nmf.r:140-141).
// ---------------------------------------------------------------------------------------------
static __global__ __launch_bounds__(NT) void k_labels(const RestartInfo* __restrict__ ri, const int* __restrict__ slot,
                                               const double* __restrict__ H, long n_pad, int n, int rule,
                                               int32_t* __restrict__ labels) {
  const int r = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int c0 = ri[r].col0, k = ri[r].k;
  int best = 0;
  double bv = H[(long)c0 * n_pad + j];
  for (int a = 1; a < k; ++a) {
    const double v = H[(long)(c0 + a) * n_pad + j];
    if (rule == 0 ? (v > bv) : (v < bv)) {
      bv = v;
      best = a;
    }
  }
  labels[(long)slot[r] * n + j] = best + 1;
}

// counts[g][i + j*n] = sum over the group's restarts of [L[i] == L[j]]
static __global__ __launch_bounds__(NT) void k_counts(const int32_t* __restrict__ labels, const int* __restrict__ grp_begin,
                                               const int* __restrict__ grp_list, int n, int32_t* __restrict__ counts) {
  const int gidx = blockIdx.z;
  const int i = blockIdx.x * 16 + (threadIdx.x & 15);
  const int j = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (i >= n || j >= n) return;
  const int b = grp_begin[gidx], e = grp_begin[gidx + 1];
  int32_t cnt = 0;
  for (int q = b; q < e; ++q) {
    const int32_t* L = labels + (long)grp_list[q] * n;
    cnt += (L[i] == L[j]);
  }
  counts[(long)gidx * n * n + (long)j * n + i] = cnt;
}

static __global__ void k_divide(const int32_t* __restrict__ counts, double denom, long len, double* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < len) out[i] = (double)counts[i] / denom;
}

// A (m x n, ld lda) -> Acm (column j at j*m_pad, zero padded) and Arm (row i at i*n_pad)
static __global__ void k_layout_a(const double* __restrict__ A, long lda, int m, int n, long m_pad, long n_pad,
                           double* __restrict__ Acm, double* __restrict__ Arm) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y;
  if (i >= m) return;
  const double v = A[(long)j * lda + i];
  Acm[(long)j * m_pad + i] = v;
  Arm[i * n_pad + j] = v;
}

// ---------------------------------------------------------------------------------------------
// calculateNorm (calculatenorm.c:44-78) and calculateMaxchange (calculatemaxchange.c:42-71)
// ---------------------------------------------------------------------------------------------
static __global__ __launch_bounds__(NT) void k_norm_partial(const double* __restrict__ a, const double* __restrict__ w,
                                                     const double* __restrict__ h, double* __restrict__ d, int m,
                                                     int n, int k, double* __restrict__ partial) {
  __shared__ double red[NT];
  const long len = (long)m * n;
  double ss = 0.0;
  for (long idx = (long)blockIdx.x * NT + threadIdx.x; idx < len; idx += (long)gridDim.x * NT) {
    const long j = idx / m, i = idx - j * m;
    double s = 0.0;
    for (int q = 0; q < k; ++q) s = fma(w[i + (long)q * m], h[q + j * k], s);
    const double v = a[idx] - s;
    d[idx] = v;
    ss = fma(v, v, ss);
  }
  red[threadIdx.x] = ss;
  __syncthreads();
  for (int off = NT / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

static __global__ __launch_bounds__(NT) void k_maxchange_partial(const double* __restrict__ mat, double* __restrict__ mat0,
                                                          long len, double* __restrict__ partial) {
  __shared__ double r0[NT], r1[NT];
  double mx0 = 0.0, mxd = 0.0;
  for (long idx = (long)blockIdx.x * NT + threadIdx.x; idx < len; idx += (long)gridDim.x * NT) {
    const double v0 = mat0[idx];
    mx0 = fmax(mx0, fabs(v0));
    const double dv = v0 - mat[idx];
    mat0[idx] = dv;
    mxd = fmax(mxd, fabs(dv));
  }
  r0[threadIdx.x] = mx0;
  r1[threadIdx.x] = mxd;
  __syncthreads();
  for (int off = NT / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      r0[threadIdx.x] = fmax(r0[threadIdx.x], r0[threadIdx.x + off]);
      r1[threadIdx.x] = fmax(r1[threadIdx.x], r1[threadIdx.x + off]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = r0[0];
    partial[2 * blockIdx.x + 1] = r1[0];
  }
}

}  // namespace nmfc
