/*
 * oracle/nmf_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * A plain-C CPU restatement of the reference's NMF restart hot path
 * (mschubert/NMFconsensus @ v1, read-only at /root/reference).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 * The product path (nmfconsensus_amd/libnmf.so) never links or calls it.
 *
 * Pinning: every function here is checked by tests/test_oracle.py against
 *   - the golden vectors in tests/golden/ (produced by the reference's own C sources,
 *     compiled out-of-tree by oracle/Makefile into oracle/_ref/, see tests/golden/make_golden.py),
 *   - glibc's own srand()/rand() for the TYPE_3 restatement.
 *
 * Conventions follow libnmf: matrices are column-major; W is m x k (ld m), H is k x n (ld k).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

/* ---------------------------------------------------------------------------------------
 * glibc TYPE_3 additive-feedback generator (what libc srand()/rand() are on this image).
 * randnumber.c:27-35 draws from it:  min + ((max - min) * rand()) / (double)RAND_MAX
 * Restated from the published algorithm: r[0]=seed (0 -> 1); r[i] = 16807 r[i-1] mod (2^31-1)
 * (Schrage form) for i = 1..30; r[i] = r[i-31] for i = 31..33; afterwards
 * r[i] = r[i-31] + r[i-3] (mod 2^32); output o_t = r[t+344] >> 1.
 * --------------------------------------------------------------------------------------- */
typedef struct orc_rand_t {
  uint32_t ring[34];
  uint64_t pos; /* index i of the next r[i] to produce */
} orc_rand_t;

void orc_srand(orc_rand_t* st, uint32_t seed) {
  uint32_t r[344];
  int32_t word = (int32_t)(seed ? seed : 1u);
  r[0] = (uint32_t)word;
  for (int i = 1; i < 31; ++i) {
    long hi = word / 127773;
    long lo = word % 127773;
    long w = 16807 * lo - 2836 * hi;
    if (w < 0) w += 2147483647;
    word = (int32_t)w;
    r[i] = (uint32_t)word;
  }
  for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
  for (int i = 34; i < 344; ++i) r[i] = r[i - 31] + r[i - 3];
  /* ring keeps r[i] at ring[i % 34] */
  for (int i = 344 - 34; i < 344; ++i) st->ring[i % 34] = r[i];
  st->pos = 344;
}

int32_t orc_rand(orc_rand_t* st) {
  uint64_t i = st->pos++;
  uint32_t v = st->ring[(i - 31) % 34] + st->ring[(i - 3) % 34];
  st->ring[i % 34] = v;
  return (int32_t)(v >> 1);
}

/* randnumber.c:34 -- (max - min) * rand() is an int product (wraps like two's complement here). */
double orc_randnumber(orc_rand_t* st, int min, int max) {
  int32_t prod = (int32_t)((uint32_t)(max - min) * (uint32_t)orc_rand(st));
  return (double)min + ((double)prod / (double)2147483647);
}

/* generatematrix.c:131-137 (init == ran): W[0..m*k) then H[0..k*n), one draw each. */
void orc_generate_ran(orc_rand_t* st, int m, int n, int k, int min, int max, double* W, double* H) {
  for (long i = 0; i < (long)m * k; ++i) W[i] = orc_randnumber(st, min, max);
  for (long i = 0; i < (long)k * n; ++i) H[i] = orc_randnumber(st, min, max);
}

/* Seeded restart init used by the batched sweep: srand(seed) then generateMatrix(ran, 0, 1). */
void orc_init_restart(uint32_t seed, int m, int n, int k, double* W, double* H) {
  orc_rand_t st;
  orc_srand(&st, seed);
  orc_generate_ran(&st, m, n, k, 0, 1, W, H);
}

/* ---------------------------------------------------------------------------------------
 * nmf_mu restatement (libnmf/nmf_mu.c:84-315)
 * --------------------------------------------------------------------------------------- */
enum { ORC_STOP_FIXED = 0, ORC_STOP_REF_COMPAT = 1, ORC_STOP_ARGMAX_STABLE = 2, ORC_STOP_TOLX = 3 };

#define ORC_DIV_BY_ZERO_AVOIDANCE 1E-09 /* nmf_mu.c:56 */

/* C[k x n] = X[m x k]^T * Y[m x n]   (dgemm('T','N') at nmf_mu.c:174 / :176) */
static void gemm_tn(int k, int n, int m, const double* X, const double* Y, double* C) {
  for (int j = 0; j < n; ++j)
    for (int a = 0; a < k; ++a) {
      const double* x = X + (long)a * m;
      const double* y = Y + (long)j * m;
      double s = 0.0;
      for (int i = 0; i < m; ++i) s += x[i] * y[i];
      C[a + (long)j * k] = s;
    }
}

/* C[p x q] = X[p x r] * Y[r x q], all column-major (dgemm('N','N') at nmf_mu.c:178 / :202) */
static void gemm_nn(int p, int q, int r, const double* X, int ldx, const double* Y, int ldy, double* C, int ldc) {
  for (int j = 0; j < q; ++j) {
    double* c = C + (long)j * ldc;
    for (int i = 0; i < p; ++i) c[i] = 0.0;
    for (int l = 0; l < r; ++l) {
      double y = Y[l + (long)j * ldy];
      const double* x = X + (long)l * ldx;
      for (int i = 0; i < p; ++i) c[i] += x[i] * y;
    }
  }
}

/* C[p x q] = X[p x r] * Y[q x r]^T  (dgemm('N','T') at nmf_mu.c:198 / :200) */
static void gemm_nt(int p, int q, int r, const double* X, int ldx, const double* Y, int ldy, double* C, int ldc) {
  for (int j = 0; j < q; ++j) {
    double* c = C + (long)j * ldc;
    for (int i = 0; i < p; ++i) c[i] = 0.0;
    for (int l = 0; l < r; ++l) {
      double y = Y[j + (long)l * ldy];
      const double* x = X + (long)l * ldx;
      for (int i = 0; i < p; ++i) c[i] += x[i] * y;
    }
  }
}

/* nmf_mu.c:184-191 / :209-216 -- note the order: add, divide, multiply; ZERO_THRESHOLD is 0.0 (common.h:15) */
static void mu_update(long len, const double* old, const double* num, const double* den, double* out) {
  for (long i = 0; i < len; ++i) {
    if (old[i] == 0. || num[i] == 0.)
      out[i] = 0.;
    else {
      double t = old[i] * (num[i] / (den[i] + ORC_DIV_BY_ZERO_AVOIDANCE));
      out[i] = (t < 0.0) ? 0. : t;
    }
  }
}

/* REF_COMPAT class of window i (nmf_mu.c:256-261): the flat buffer h0 is read at h0[i*n + j] for
 * j in [0,k); indices at or beyond k*n read the caller's zero padding ("REF_COMPAT"). */
static int refcompat_class(const double* h, int k, int n, int i) {
  int best = 0;
  long base = (long)i * n;
  for (int j = 1; j < k; ++j) {
    long a = base + j, b = base + j - 1;
    double va = (a < (long)k * n) ? h[a] : 0.0;
    double vb = (b < (long)k * n) ? h[b] : 0.0;
    if (va > vb) best = j;
  }
  return best;
}

/* first index of the maximum of column j of H (k x n) */
static int argmax_col(const double* h, int k, int j) {
  int best = 0;
  for (int a = 1; a < k; ++a)
    if (h[a + (long)j * k] > h[best + (long)j * k]) best = a;
  return best;
}

/*
 * Runs the MU loop on W (m x k) and H (k x n) in place.  Returns the number of iterations run
 * (the value nmf_mu writes to *maxiter on early exit, nmf_mu.c:270; maxiter otherwise).
 * Results are always left in W/H (the reference leaves them in the caller's buffers only for an
 * even iteration count, nmf_mu.c:241-242 -- a safe superset).
 */
int orc_nmf_mu(const double* A, double* W, double* H, int m, int n, int k, int maxiter, int stop_rule) {
  double* numerh = (double*)malloc(sizeof(double) * k * n);
  double* work1 = (double*)malloc(sizeof(double) * k * k);
  double* work2 = (double*)malloc(sizeof(double) * k * n);
  double* h = (double*)malloc(sizeof(double) * k * n);
  double* numerw = (double*)malloc(sizeof(double) * m * k);
  double* work2w = (double*)malloc(sizeof(double) * m * k);
  double* w = (double*)malloc(sizeof(double) * m * k);
  int* classes = (int*)calloc(n > 0 ? n : 1, sizeof(int)); /* nmf_mu.c:132, zero-initialised */
  int unchanged = 0;                                         /* nmf_mu.c:133 */
  int iter, ran = maxiter;
  for (iter = 1; iter <= maxiter; ++iter) {
    gemm_tn(k, n, m, W, A, numerh);                       /* :174 numerh = W^T A */
    gemm_tn(k, k, m, W, W, work1);                        /* :176 work1 = W^T W */
    gemm_nn(k, n, k, work1, k, H, k, work2, k);           /* :178 work2 = work1 H */
    mu_update((long)k * n, H, numerh, work2, h);          /* :184-191 */
    gemm_nt(m, k, n, A, m, h, k, numerw, m);              /* :198 numerw = A h^T */
    gemm_nt(k, k, n, h, k, h, k, work1, k);               /* :200 work1 = h h^T */
    gemm_nn(m, k, k, W, m, work1, k, work2w, m);          /* :202 work2w = W work1 */
    mu_update((long)m * k, W, numerw, work2w, w);         /* :209-216 */
    memcpy(W, w, sizeof(double) * m * k);                 /* :241-242 swap */
    memcpy(H, h, sizeof(double) * k * n);
    if (stop_rule != ORC_STOP_FIXED && iter > 1 && iter % 2 == 0) { /* :253 */
      int same = 1;
      int nwin = (stop_rule == ORC_STOP_REF_COMPAT) ? (k < n ? k : n) : n;
      for (int i = 0; i < nwin; ++i) {
        int c = (stop_rule == ORC_STOP_REF_COMPAT) ? refcompat_class(H, k, n, i) : argmax_col(H, k, i);
        if (classes[i] != c) {
          same = 0;
          classes[i] = c;
        }
      }
      if (same) {
        if (++unchanged >= 200) { /* :269 */
          ran = iter;
          break;
        }
      } else {
        unchanged = 0;
      }
    }
  }
  free(numerh); free(work1); free(work2); free(h); free(numerw); free(work2w); free(w); free(classes);
  return ran;
}

/* Cluster labels of one restart, 1-based like R.
 * rule 0 (ARGMAX): first index of the column maximum (documented intent, nmf.r:127 comment).
 * rule 1 (R_ORDER): apply(H, 2, order)[1,] at nmf.r:128 = first index of the column minimum. */
void orc_labels(const double* H, int k, int n, int rule, int32_t* labels) {
  for (int j = 0; j < n; ++j) {
    const double* c = H + (long)j * k;
    int best = 0;
    for (int a = 1; a < k; ++a) {
      if (rule == 0 ? (c[a] > c[best]) : (c[a] < c[best])) best = a;
    }
    labels[j] = best + 1;
  }
}

/* nmf.r:140-141 connectivity counts: counts[i + j*n] += (l_r[i] == l_r[j]) over R restarts. */
void orc_counts(const int32_t* labels, int R, int n, int32_t* counts) {
  memset(counts, 0, sizeof(int32_t) * n * n);
  for (int r = 0; r < R; ++r) {
    const int32_t* l = labels + (long)r * n;
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) counts[i + (long)j * n] += (l[i] == l[j]);
  }
}

/* calculatenorm.c:44-78: ||A - W H||_F / sqrt(m n)  (d receives A - W H) */
double orc_calculate_norm(const double* a, const double* w, const double* h, double* d, int m, int n, int k) {
  double ss = 0.0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) {
      double s = 0.0;
      for (int l = 0; l < k; ++l) s += w[i + (long)l * m] * h[l + (long)j * k];
      double v = a[i + (long)j * m] - s;
      d[i + (long)j * m] = v;
      ss += v * v;
    }
  return sqrt(ss) / sqrt((double)m * n);
}

/* calculatemaxchange.c:42-71: max|mat0 - mat| / (sqrteps + max|mat0|); side effect mat0 -= mat */
double orc_calculate_maxchange(const double* mat, double* mat0, int m, int n, double sqrteps) {
  double mx0 = 0.0, mxd = 0.0;
  long len = (long)m * n;
  for (long i = 0; i < len; ++i) {
    double v = fabs(mat0[i]);
    if (v > mx0 || isnan(v)) mx0 = v;
  }
  for (long i = 0; i < len; ++i) {
    mat0[i] = mat0[i] - mat[i];
    double v = fabs(mat0[i]);
    if (v > mxd || isnan(v)) mxd = v;
  }
  return mxd / (sqrteps + mx0);
}

/*
 * The MU update (nmf_mu.c:174-216) under libnmf's TolX/TolFun convergence test as nmf_als.c:304-349
 * writes it: after each iteration dnorm = calculateNorm(A, W, H) (:304), dw / dh = calculateMaxchange
 * of the new vs the previous factor (:310, :316), delta = max(dh, dw), dnorm0 = dnorm (:330); on even
 * iterations > 1 stop if delta < TolX, else if dnorm <= TolFun * dnorm0 (:341-349).  Returns the
 * iteration count.  sqrteps = sqrt(dlamch('E')) = 2^-26.5.
 */
int orc_nmf_mu_tol(const double* A, double* W, double* H, int m, int n, int k, int maxiter, double TolX,
                   double TolFun) {
  const double sqrteps = 1.0536712127723509e-08;
  double* W0 = (double*)malloc(sizeof(double) * (size_t)m * k);
  double* H0 = (double*)malloc(sizeof(double) * (size_t)k * n);
  double* d = (double*)malloc(sizeof(double) * (size_t)m * n);
  int ran = maxiter;
  for (int iter = 1; iter <= maxiter; ++iter) {
    memcpy(W0, W, sizeof(double) * (size_t)m * k);
    memcpy(H0, H, sizeof(double) * (size_t)k * n);
    orc_nmf_mu(A, W, H, m, n, k, 1, ORC_STOP_FIXED);
    const double dnorm = orc_calculate_norm(A, W, H, d, m, n, k);
    const double dw = orc_calculate_maxchange(W, W0, m, k, sqrteps);
    const double dh = orc_calculate_maxchange(H, H0, k, n, sqrteps);
    const double delta = (dh > dw) ? dh : dw;
    const double dnorm0 = dnorm;
    if (iter > 1 && iter % 2 == 0) {
      if (delta < TolX) {
        ran = iter;
        break;
      } else if (dnorm <= TolFun * dnorm0) {
        ran = iter;
        break;
      }
    }
  }
  free(W0);
  free(H0);
  free(d);
  return ran;
}
