/*
 * examples/c_sweep.c -- the library from plain C99, the way a C host (or R's .C) drives it: no torch, no Python.
 *
 *   1. nmfc_sweep: the whole k-sweep (nmf.r:53-70, 106-143) on a planted 1000 x 40 matrix, k = 2..5, 5 restarts
 *      each (test_nmf.r's job shape), libnmf init stream, the reference's stop rule; then nmfc_cophenetic_batch
 *      (nmf.r:165-172) per k.
 *   2. The drop-in: generateMatrix(ran) + nmf_mu (nmf.r:37-45 with the libnmf init) for one restart of k = 3.
 *
 * Build (examples/Makefile, also run by __graft_entry__.build()):
 *   gcc -std=c99 -O2 -Wall -Wextra -pedantic -Iinclude examples/c_sweep.c -Lnmfconsensus_amd/lib -lnmf -o examples/c_sweep
 * Run: examples/c_sweep [out_dir]   -- out_dir receives A.bin (m x n fp64, column-major), counts.bin (nk x n x n
 * int32), iters.bin (jobs int32) and nmf_mu.bin (the drop-in's W then H, fp64) for tests/test_gpu_c_consumer.py.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "libnmf_compat.h"
#include "nmfc.h"

/* splitmix64 -> uniform [0, 1) (53 bits): deterministic, so the test can rebuild the same A */
static uint64_t sm_state = 20261015u;
static double unif(void) {
  uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

static int write_bin(const char* dir, const char* name, const void* p, size_t bytes) {
  char path[4096];
  FILE* f;
  snprintf(path, sizeof path, "%s/%s", dir, name);
  f = fopen(path, "wb");
  if (!f || fwrite(p, 1, bytes, f) != bytes) {
    fprintf(stderr, "cannot write %s\n", path);
    if (f) fclose(f);
    return -1;
  }
  return fclose(f);
}

int main(int argc, char** argv) {
  const int m = 1000, n = 40, ks[] = {2, 3, 4, 5}, nk = 4, R = 5, njobs = nk * R;
  const char* out_dir = argc > 1 ? argv[1] : NULL;
  double* A = malloc(sizeof(double) * m * n);
  int32_t* counts = malloc(sizeof(int32_t) * nk * n * n);
  double* cons = malloc(sizeof(double) * nk * n * n);
  int32_t* iters = malloc(sizeof(int32_t) * njobs);
  double rho[4];
  nmfc_sweep_opts o;
  nmfc_result r;
  int i, j, q, rc;
  long long total = 0;
  if (!A || !counts || !cons || !iters) return 2;

  /* planted two-group matrix: genes 0..499 high in samples 0..19, genes 500..999 high in 20..39, plus noise */
  for (j = 0; j < n; ++j)
    for (i = 0; i < m; ++i) A[(size_t)j * m + i] = 0.1 + unif() + (((i < m / 2) == (j < n / 2)) ? 2.0 : 0.0);

  nmfc_default_opts(&o);                 /* maxiter 10000, REF_COMPAT stop rule, seed 123, libnmf init */
  memset(&r, 0, sizeof r);
  r.counts = counts;
  r.consensus = cons;
  r.iters = iters;
  rc = nmfc_sweep(A, m, n, ks, nk, R, &o, &r);
  if (rc != 0) {
    fprintf(stderr, "nmfc_sweep: %s\n", nmfc_last_error());
    return 1;
  }
  for (j = 0; j < njobs; ++j) total += iters[j];
  if (nmfc_cophenetic_batch(cons, nk, n, 0, rho, NULL, NULL, NULL) != 0) {
    fprintf(stderr, "nmfc_cophenetic_batch: %s\n", nmfc_last_error());
    return 1;
  }
  printf("%s: %d jobs, %lld restart-iterations, max %d, %.2f ms\n", nmfc_version(), njobs, total, r.max_iter_run,
         1e3 * r.seconds_total);
  for (q = 0; q < nk; ++q) printf("k=%d cophenetic rho %.6f\n", ks[q], rho[q]);

  /* the drop-in, as nmf.r calls it: generateMatrix(ran) after srand(seed), then .C("nmf_mu", ...) */
  {
    int mm = m, nn = n, k = 3, maxiter = 10000, mn = 0, mx = 1;
    const double tolx = 1e-4, tolfun = 1e-4;
    init_t init = ran;
    options_t opts;
    double* W = malloc(sizeof(double) * m * k);
    double* H = malloc(sizeof(double) * k * n);
    if (!W || !H) return 2;
    set_default_opts(&opts);
    (void)randnumber(0, 1);              /* the reference's first call seeds from the clock ... */
    srand(123);                          /* ... then the job seed */
    generateMatrix(&mm, &nn, &k, &init, &mn, &mx, W, H, A, &opts);
    if (nmf_mu(A, W, H, &mm, &nn, &k, &maxiter, &tolx, &tolfun) != 0) {
      fprintf(stderr, "nmf_mu failed\n");
      return 1;
    }
    printf("nmf_mu k=%d: stopped at iteration %d\n", k, maxiter);
    if (out_dir) {
      double* wh = malloc(sizeof(double) * (m * k + k * n + 1));
      if (!wh) return 2;
      memcpy(wh, W, sizeof(double) * m * k);
      memcpy(wh + m * k, H, sizeof(double) * k * n);
      wh[m * k + k * n] = (double)maxiter;
      if (write_bin(out_dir, "nmf_mu.bin", wh, sizeof(double) * (m * k + k * n + 1))) return 1;
      free(wh);
    }
    free(W);
    free(H);
  }
  if (out_dir && (write_bin(out_dir, "A.bin", A, sizeof(double) * m * n) ||
                  write_bin(out_dir, "counts.bin", counts, sizeof(int32_t) * nk * n * n) ||
                  write_bin(out_dir, "iters.bin", iters, sizeof(int32_t) * njobs)))
    return 1;
  free(A);
  free(counts);
  free(cons);
  free(iters);
  return 0;
}
