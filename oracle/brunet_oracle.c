/*
 * oracle/brunet_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C CPU restatement of the Brunet KL-divergence multiplicative-update NMF that the BROAD
 * `nmfconsensus(...)` R script runs per restart (BASELINE.json configs[4]).
 * The reference repository only names that script (commented-out call at test_nmf.r:29); its source
 * is NOT in /root/reference, so this is restated from the published algorithm:
 *   Brunet, Tamayo, Golub, Mesirov (2004) PNAS 101:4164, "Metagenes and molecular pattern
 *   discovery using matrix factorization", and GenePattern's NMFConsensus module (function NMF.div):
 *     VP <- W %*% H;  H <- H * (t(W) %*% (V/VP)) + eps;  H[i,] <- H[i,] / colSums(W)[i]
 *     VP <- W %*% H;  W <- W * ((V/VP) %*% t(H)) + eps;  W[,i] <- W[,i] / rowSums(H)[i]
 *     every stopfreq iterations: membership[j] = order(H[,j], decreasing=TRUE)[1]; stop after
 *     stopconv consecutive unchanged checks.  eps = .Machine$double.eps = 2^-52.
 *   Init: set.seed(seed); W <- matrix(runif(m*k), m, k); H <- matrix(runif(k*n), k, n).
 * PARITY UNPINNED against the reference (neither the script nor R exists in the image); the R
 * Mersenne-Twister restatement below IS pinned by R's published set.seed()/runif() values
 * (tests/test_brunet_oracle.py).
 *
 * Conventions: column-major, W m x k (ld m), H k x n (ld k).  Matrix products accumulate in the
 * reference-BLAS dgemm order (sequential over the inner index); R's sum() accumulates in long double.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

/* ---------------------------------------------------------------------------------------
 * R's default RNG: Mersenne-Twister MT19937 (Matsumoto & Nishimura 1998) with R's seeding.
 * set.seed(s): s is scrambled by 50 steps of s <- 69069 s + 1 (mod 2^32); the next 625 LCG
 * outputs fill the seed vector whose element 0 is the position `mti` (reset to 624, so the first
 * draw regenerates the block) and elements 1..624 the state.  runif(): tempered 32-bit word
 * times 2^-32, pushed into (0,1) (values of exactly 0 or 1 are replaced by 2^-33 / 1 - 2^-33).
 * --------------------------------------------------------------------------------------- */
typedef struct orc_rmt_t {
  uint32_t mt[624];
  int mti;
} orc_rmt_t;

void orc_rmt_seed(orc_rmt_t* st, uint32_t seed) {
  for (int j = 0; j < 50; ++j) seed = 69069u * seed + 1u;
  seed = 69069u * seed + 1u; /* element 0 of the seed vector (mti), overwritten below */
  for (int j = 0; j < 624; ++j) {
    seed = 69069u * seed + 1u;
    st->mt[j] = seed;
  }
  st->mti = 624;
}

static void rmt_twist(uint32_t* mt) {
  const uint32_t UP = 0x80000000u, LO = 0x7fffffffu, MA = 0x9908b0dfu;
  int kk;
  uint32_t y;
  for (kk = 0; kk < 624 - 397; ++kk) {
    y = (mt[kk] & UP) | (mt[kk + 1] & LO);
    mt[kk] = mt[kk + 397] ^ (y >> 1) ^ ((y & 1u) ? MA : 0u);
  }
  for (; kk < 623; ++kk) {
    y = (mt[kk] & UP) | (mt[kk + 1] & LO);
    mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ ((y & 1u) ? MA : 0u);
  }
  y = (mt[623] & UP) | (mt[0] & LO);
  mt[623] = mt[396] ^ (y >> 1) ^ ((y & 1u) ? MA : 0u);
}

double orc_rmt_unif(orc_rmt_t* st) {
  if (st->mti >= 624) {
    rmt_twist(st->mt);
    st->mti = 0;
  }
  uint32_t y = st->mt[st->mti++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  const double i2_32m1 = 2.328306437080797e-10; /* 1 / (2^32 - 1) */
  double v = (double)y * 2.3283064365386963e-10;
  if (v <= 0.0) return 0.5 * i2_32m1;
  if (1.0 - v <= 0.0) return 1.0 - 0.5 * i2_32m1;
  return v;
}

/* set.seed(seed); W <- matrix(runif(m*k), m, k); H <- matrix(runif(k*n), k, n) */
void orc_brunet_init(uint32_t seed, int m, int n, int k, double* W, double* H) {
  orc_rmt_t st;
  orc_rmt_seed(&st, seed);
  for (long i = 0; i < (long)m * k; ++i) W[i] = orc_rmt_unif(&st);
  for (long i = 0; i < (long)k * n; ++i) H[i] = orc_rmt_unif(&st);
}

/* membership[j] = order(H[,j], decreasing = TRUE)[1]: the first row of the column maximum, 1-based */
static int first_max_row(const double* H, int k, int j) {
  int best = 0;
  for (int c = 1; c < k; ++c)
    if (H[(long)j * k + c] > H[(long)j * k + best]) best = c;
  return best + 1;
}

/* NMF.div: returns the iteration count t (the loop index at the break, or maxiter).
 * err (optional, maxiter entries): error.v[t] = sum(V*log((V+eps)/(VP+eps)) - V + VP)/(m n). */
int orc_brunet(const double* A, double* W, double* H, int m, int n, int k, int maxiter, int stopconv,
               int stopfreq, double* err) {
  const double eps = 2.220446049250313e-16; /* .Machine$double.eps */
  double* VP = (double*)malloc(sizeof(double) * (size_t)m * n);
  double* Q = (double*)malloc(sizeof(double) * (size_t)m * n);
  double* G = (double*)malloc(sizeof(double) * (size_t)k * n);
  double* F = (double*)malloc(sizeof(double) * (size_t)m * k);
  double* norm = (double*)malloc(sizeof(double) * (size_t)k);
  int* newm = (int*)calloc((size_t)n, sizeof(int));
  int* oldm = (int*)calloc((size_t)n, sizeof(int));
  int nochange = 0, t;
  for (t = 1; t <= maxiter; ++t) {
    /* VP = W %*% H ; Q = V / VP */
    for (int j = 0; j < n; ++j) {
      for (int i = 0; i < m; ++i) VP[(long)j * m + i] = 0.0;
      for (int l = 0; l < k; ++l) {
        const double h = H[(long)j * k + l];
        for (int i = 0; i < m; ++i) VP[(long)j * m + i] += h * W[(long)l * m + i];
      }
      for (int i = 0; i < m; ++i) Q[(long)j * m + i] = A[(long)j * m + i] / VP[(long)j * m + i];
    }
    /* G = t(W) %*% Q */
    for (int j = 0; j < n; ++j)
      for (int c = 0; c < k; ++c) {
        double s = 0.0;
        for (int i = 0; i < m; ++i) s += W[(long)c * m + i] * Q[(long)j * m + i];
        G[(long)j * k + c] = s;
      }
    /* norm = apply(W, 2, sum) */
    for (int c = 0; c < k; ++c) {
      long double s = 0.0L;
      for (int i = 0; i < m; ++i) s += W[(long)c * m + i];
      norm[c] = (double)s;
    }
    for (long e = 0; e < (long)k * n; ++e) {
      const double v = H[e] * G[e];
      H[e] = (v + eps) / norm[e % k];
    }
    /* VP = W %*% H (old W, new H) ; Q = V / VP */
    for (int j = 0; j < n; ++j) {
      for (int i = 0; i < m; ++i) VP[(long)j * m + i] = 0.0;
      for (int l = 0; l < k; ++l) {
        const double h = H[(long)j * k + l];
        for (int i = 0; i < m; ++i) VP[(long)j * m + i] += h * W[(long)l * m + i];
      }
      for (int i = 0; i < m; ++i) Q[(long)j * m + i] = A[(long)j * m + i] / VP[(long)j * m + i];
    }
    /* F = Q %*% t(H) */
    for (int c = 0; c < k; ++c) {
      for (int i = 0; i < m; ++i) F[(long)c * m + i] = 0.0;
      for (int j = 0; j < n; ++j) {
        const double h = H[(long)j * k + c];
        for (int i = 0; i < m; ++i) F[(long)c * m + i] += Q[(long)j * m + i] * h;
      }
    }
    /* norm = apply(H, 1, sum) */
    for (int c = 0; c < k; ++c) {
      long double s = 0.0L;
      for (int j = 0; j < n; ++j) s += H[(long)j * k + c];
      norm[c] = (double)s;
    }
    for (long e = 0; e < (long)m * k; ++e) {
      const double v = W[e] * F[e];
      W[e] = (v + eps) / norm[e / m];
    }
    if (err) {
      long double s = 0.0L;
      for (long e = 0; e < (long)m * n; ++e) {
        const double v = A[e], p = VP[e];
        s += v * log((v + eps) / (p + eps)) - v + p;
      }
      err[t - 1] = (double)(s / ((long double)m * n));
    }
    if (t % stopfreq == 0) {
      int same = 0;
      for (int j = 0; j < n; ++j) {
        newm[j] = first_max_row(H, k, j);
        same += newm[j] == oldm[j];
      }
      nochange = same == n ? nochange + 1 : 0;
      if (nochange == stopconv) break;
      memcpy(oldm, newm, sizeof(int) * (size_t)n);
    }
  }
  if (t > maxiter) t = maxiter;
  free(VP);
  free(Q);
  free(G);
  free(F);
  free(norm);
  free(newm);
  free(oldm);
  return t;
}
