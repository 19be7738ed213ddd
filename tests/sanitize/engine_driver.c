/* Host-sanitizer driver for the engine's host code on a real GPU (test infrastructure).  tests/sanitize/Makefile
 * links it twice: against the product libnmf.so and against a libnmf built with every host side under
 * -Xarch_host -fsanitize=address,undefined (device code is not instrumented; the pool runs no GPU sanitizer).
 * tests/test_gpu_host_asan.py runs both on the GPU and requires identical output files, a zero exit and no sanitizer
 * report.  What it drives, all through the C ABI (include/nmfc.h, include/libnmf_compat.h):
 *   1. nmfc_sweep on a 1000 x 40 matrix, k = 2..9, R = 5: the small-shape path (solo kernels, k_small_mu block);
 *   2. one engine, two runs on a 2048 x 96 matrix, k = 2..10, R = 8, REF_COMPAT then ARGMAX_STABLE: the MFMA
 *      engine's packing, repacks, tile choices, narrow tail kernels and stop polling, the engine reused;
 *   3. a sharded run (jobs 10..50) of the same engine with caller-provided W / H init and every result array;
 *   4. the drop-in nmf_mu for k = 2..5 on the 1000 x 40 matrix (solo, team) and k = 1, 17 on 300 x 40 (generic);
 *   5. a Brunet sweep, k = 2..4, R = 4, 400 x 30;
 *   6. nmfc_cophenetic_batch on the consensus of run 2;
 *   7. two host threads, each with an engine of its own over the same matrix, running job shards concurrently (the
 *      restart groups of distributed.RestartGroups, from C): their counts sum to the one-engine run's.
 * Output: argv[1]/engine_driver.bin (counts, iterations, W / H digests) -- the two builds must agree bit for bit. */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "libnmf_compat.h"
#include "nmfc.h"

static uint64_t sm_state = 7u;
static double unif(void) {
  uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

static double* planted(int m, int n, int groups) {
  double* A = malloc(sizeof(double) * (size_t)m * n);
  int i, j;
  if (!A) return NULL;
  for (j = 0; j < n; ++j)
    for (i = 0; i < m; ++i) A[(size_t)j * m + i] = 0.1 + unif() + ((i * groups / m) == (j * groups / n) ? 2.0 : 0.0);
  return A;
}

static FILE* out;
static void put(const void* p, size_t bytes) { fwrite(p, 1, bytes, out); }

static int fail(const char* what) {
  fprintf(stderr, "FAIL %s: %s\n", what, nmfc_last_error());
  return 1;
}

static int sweep_small(void) {
  const int m = 1000, n = 40, ks[] = {2, 3, 4, 5, 6, 7, 8, 9}, nk = 8, R = 5;
  double* A = planted(m, n, 2);
  int32_t* counts = malloc(sizeof(int32_t) * nk * n * n);
  int32_t* iters = malloc(sizeof(int32_t) * nk * R);
  nmfc_sweep_opts o;
  nmfc_result r;
  if (!A || !counts || !iters) return fail("alloc");
  nmfc_default_opts(&o);
  memset(&r, 0, sizeof r);
  r.counts = counts;
  r.iters = iters;
  if (nmfc_sweep(A, m, n, ks, nk, R, &o, &r) != 0) return fail("nmfc_sweep small");
  put(counts, sizeof(int32_t) * nk * n * n);
  put(iters, sizeof(int32_t) * nk * R);
  free(A);
  free(counts);
  free(iters);
  return 0;
}

static int engine_runs(void) {
  const int m = 2048, n = 96, ks[] = {2, 3, 4, 5, 6, 7, 8, 9, 10}, nk = 9, R = 8, nj = nk * R;
  const int rules[2] = {NMFC_STOP_REF_COMPAT, NMFC_STOP_ARGMAX_STABLE};
  double* A = planted(m, n, 3);
  int32_t* counts = malloc(sizeof(int32_t) * nk * n * n);
  double* cons = malloc(sizeof(double) * nk * n * n);
  int32_t* iters = malloc(sizeof(int32_t) * nj);
  int32_t* labels = malloc(sizeof(int32_t) * nj * n);
  int32_t* early = malloc(sizeof(int32_t) * nj);
  double rho[9];
  nmfc_engine* e;
  nmfc_sweep_opts o;
  nmfc_result r;
  int q, j, b = 10, t = 50;
  size_t wsz = 0, hsz = 0;
  double *W0, *H0, *W, *H;
  if (!A || !counts || !cons || !iters || !labels || !early) return fail("alloc");
  e = nmfc_engine_create(-1, A, m, n, 0);
  if (!e) return fail("nmfc_engine_create");
  for (q = 0; q < 2; ++q) {
    nmfc_default_opts(&o);
    o.stop_rule = rules[q];
    o.maxiter = 3000;
    memset(&r, 0, sizeof r);
    r.counts = counts;
    r.consensus = cons;
    r.iters = iters;
    r.labels = labels;
    r.stopped_early = early;
    if (nmfc_engine_run(e, ks, nk, R, &o, NULL, NULL, &r) != 0) return fail("nmfc_engine_run");
    put(counts, sizeof(int32_t) * nk * n * n);
    put(iters, sizeof(int32_t) * nj);
    put(labels, sizeof(int32_t) * nj * n);
    put(early, sizeof(int32_t) * nj);
  }
  if (nmfc_cophenetic_batch(cons, nk, n, 0, rho, NULL, NULL, NULL) != 0) return fail("nmfc_cophenetic_batch");
  put(rho, sizeof rho);
  /* a shard of the job list with the caller's init and every per-job output */
  for (j = b; j < t; ++j) {
    const int k = ks[j % nk];
    wsz += (size_t)m * k;
    hsz += (size_t)k * n;
  }
  W0 = malloc(sizeof(double) * wsz);
  H0 = malloc(sizeof(double) * hsz);
  W = malloc(sizeof(double) * wsz);
  H = malloc(sizeof(double) * hsz);
  if (!W0 || !H0 || !W || !H) return fail("alloc");
  for (size_t i = 0; i < wsz; ++i) W0[i] = 0.01 + unif();
  for (size_t i = 0; i < hsz; ++i) H0[i] = 0.01 + unif();
  nmfc_default_opts(&o);
  o.job_begin = b;
  o.job_end = t;
  memset(&r, 0, sizeof r);
  r.counts = counts;
  r.iters = iters;
  r.labels = labels;
  r.stopped_early = early;
  r.W = W;
  r.H = H;
  if (nmfc_engine_run(e, ks, nk, R, &o, W0, H0, &r) != 0) return fail("nmfc_engine_run shard");
  put(counts, sizeof(int32_t) * nk * n * n);
  put(iters, sizeof(int32_t) * (t - b));
  put(W, sizeof(double) * wsz);
  put(H, sizeof(double) * hsz);
  nmfc_engine_destroy(e);
  free(A); free(counts); free(cons); free(iters); free(labels); free(early); free(W0); free(H0); free(W); free(H);
  return 0;
}

static int dropin(void) {
  const int shapes[6][3] = {{1000, 40, 2}, {1000, 40, 3}, {1000, 40, 4}, {1000, 40, 5}, {300, 40, 1}, {300, 40, 17}};
  const double tolx = 1e-4, tolfun = 1e-4;
  int s;
  for (s = 0; s < 6; ++s) {
    int m = shapes[s][0], n = shapes[s][1], k = shapes[s][2], maxiter = 2000, lo = 0, hi = 1;
    init_t init = ran;
    options_t opts;
    double* A = planted(m, n, 2);
    double* W = malloc(sizeof(double) * m * k);
    double* H = malloc(sizeof(double) * k * n);
    if (!A || !W || !H) return fail("alloc");
    set_default_opts(&opts);
    (void)randnumber(0, 1);
    srand(123 + s);
    generateMatrix(&m, &n, &k, &init, &lo, &hi, W, H, A, &opts);
    if (nmf_mu(A, W, H, &m, &n, &k, &maxiter, &tolx, &tolfun) != 0) return fail("nmf_mu");
    put(&maxiter, sizeof maxiter);
    put(W, sizeof(double) * m * k);
    put(H, sizeof(double) * k * n);
    free(A);
    free(W);
    free(H);
  }
  nmfc_nmf_mu_release();
  return 0;
}

static int brunet(void) {
  const int m = 400, n = 30, ks[] = {2, 3, 4}, nk = 3, R = 4;
  double* A = planted(m, n, 2);
  int32_t* counts = malloc(sizeof(int32_t) * nk * n * n);
  int32_t* iters = malloc(sizeof(int32_t) * nk * R);
  nmfc_brunet_opts o;
  nmfc_result r;
  nmfc_brunet* e;
  if (!A || !counts || !iters) return fail("alloc");
  e = nmfc_brunet_create(-1, A, m, n, 0);
  if (!e) return fail("nmfc_brunet_create");
  nmfc_brunet_default_opts(&o);
  o.maxiter = 400;
  memset(&r, 0, sizeof r);
  r.counts = counts;
  r.iters = iters;
  if (nmfc_brunet_run(e, ks, nk, R, &o, NULL, NULL, &r) != 0) return fail("nmfc_brunet_run");
  put(counts, sizeof(int32_t) * nk * n * n);
  put(iters, sizeof(int32_t) * nk * R);
  nmfc_brunet_destroy(e);
  free(A);
  free(counts);
  free(iters);
  return 0;
}

struct group_arg {
  const double* A;
  int m, n, begin, end, rc;
  int32_t* counts;
};

static void* group_run(void* p) {
  struct group_arg* g = (struct group_arg*)p;
  const int ks[] = {2, 3, 4, 5, 6, 7, 8, 9, 10};
  nmfc_sweep_opts o;
  nmfc_result r;
  nmfc_engine* e = nmfc_engine_create(-1, g->A, g->m, g->n, 0);
  g->rc = 1;
  if (!e) return NULL;
  nmfc_default_opts(&o);
  o.maxiter = 3000;
  o.job_begin = g->begin;
  o.job_end = g->end;
  memset(&r, 0, sizeof r);
  r.counts = g->counts;
  g->rc = nmfc_engine_run(e, ks, 9, 8, &o, NULL, NULL, &r);
  nmfc_engine_destroy(e);
  return NULL;
}

static int groups(void) {
  const int m = 2048, n = 96, nk = 9, R = 8, nj = nk * R;
  const int ks[] = {2, 3, 4, 5, 6, 7, 8, 9, 10};
  double* A;
  int32_t *whole = malloc(sizeof(int32_t) * nk * n * n), *c0 = malloc(sizeof(int32_t) * nk * n * n),
          *c1 = malloc(sizeof(int32_t) * nk * n * n);
  struct group_arg g[2];
  pthread_t th[2];
  nmfc_sweep_opts o;
  nmfc_result r;
  long i;
  int t;
  sm_state = 99u;
  A = planted(m, n, 3);
  if (!A || !whole || !c0 || !c1) return fail("alloc");
  nmfc_default_opts(&o);
  o.maxiter = 3000;
  memset(&r, 0, sizeof r);
  r.counts = whole;
  if (nmfc_sweep(A, m, n, ks, nk, R, &o, &r) != 0) return fail("nmfc_sweep whole");
  for (t = 0; t < 2; ++t) {
    g[t].A = A;
    g[t].m = m;
    g[t].n = n;
    g[t].begin = t ? nj / 2 : 0;
    g[t].end = t ? nj : nj / 2;
    g[t].counts = t ? c1 : c0;
    if (pthread_create(&th[t], NULL, group_run, &g[t])) return fail("pthread_create");
  }
  for (t = 0; t < 2; ++t) pthread_join(th[t], NULL);
  if (g[0].rc || g[1].rc) return fail("group run");
  for (i = 0; i < (long)nk * n * n; ++i)
    if (c0[i] + c1[i] != whole[i]) {
      fprintf(stderr, "FAIL groups: counts[%ld] %d + %d != %d\n", i, c0[i], c1[i], whole[i]);
      return 1;
    }
  put(whole, sizeof(int32_t) * nk * n * n);
  free(A);
  free(whole);
  free(c0);
  free(c1);
  return 0;
}

int main(int argc, char** argv) {
  char path[4096];
  if (argc < 2) return 2;
  snprintf(path, sizeof path, "%s/engine_driver.bin", argv[1]);
  out = fopen(path, "wb");
  if (!out) return 2;
  if (sweep_small() || engine_runs() || dropin() || brunet() || groups()) return 1;
  fclose(out);
  printf("engine driver ok\n");
  return 0;
}
