/* Host-sanitizer driver for the drop-in's host C (csrc/compat.hip: setdefaultopts.c / checkarguments.c /
 * checkmatrices.c / randnumber.c / generatematrix.c restated), linked against a libnmf built with
 * -Xarch_host -fsanitize=address,undefined by tests/test_host_sanitizers.py (test infrastructure).  CPU only: no entry
 * point here touches the GPU.  Writes generateMatrix's W and H for srand(123) at 1000 x 40, k = 2..5 to argv[1]
 * (compared by the test against the reference's golden init) and exits 0 when every predicate answers as the
 * reference's does. */
#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/libnmf_compat.h"

static int fail(const char* what) {
  printf("FAIL %s\n", what);
  return 1;
}

int main(int argc, char** argv) {
  if (argc < 2) return fail("usage: compat_driver <out.bin>");
  options_t o;
  set_default_opts(&o);
  if (o.rep != 1 || o.init != ran || o.min_init != 0 || o.max_init != 1 || o.TolX != 1.0E-04) return fail("defaults");
  const char a = 'a';
  if (checkArguments(&a, 2, 10, NULL, NULL, &o) != 0) return fail("checkArguments valid");
  if (checkArguments(NULL, 2, 10, NULL, NULL, &o) != 1) return fail("checkArguments a = NULL");
  if (checkArguments(&a, -1, 10, NULL, NULL, &o) != 1) return fail("checkArguments k < 0");
  if (checkArguments(&a, 2, 10, "", NULL, &o) != 1) return fail("checkArguments empty w0 name");
  o.TolFun = -1.0;
  if (checkArguments(&a, 2, 10, NULL, NULL, &o) != 1) return fail("checkArguments TolFun < 0");
  set_default_opts(&o);

  double A[6] = {1, 2, 3, 4, 5, 6}, W[4] = {1, 1, 1, 1}, H[6] = {1, 1, 1, 1, 1, 1};
  if (checkMatrices(A, W, H, 2, 3, 2) != 0) return fail("checkMatrices valid");
  A[5] = -1.0;
  if (checkMatrices(A, W, H, 2, 3, 2) != 1) return fail("checkMatrices negative a");
  A[5] = 6.0;
  W[3] = -0.5;
  if (checkMatrices(A, W, H, 2, 3, 2) != 1) return fail("checkMatrices negative w");
  W[3] = 1.0;
  H[0] = NAN;   /* NaN fails the >= 0 scan like the reference's loop */
  if (checkMatrices(A, W, H, 2, 3, 2) != 1) return fail("checkMatrices NaN h");

  FILE* f = fopen(argv[1], "wb");
  if (!f) return fail("open output");
  const int m = 1000, n = 40, lo = 0, hi = 1;
  for (int k = 2; k <= 5; ++k) {
    double* w = malloc(sizeof(double) * m * k);
    double* h = malloc(sizeof(double) * k * n);
    if (!w || !h) return fail("malloc");
    init_t init = ran;
    errno = 0;
    srand(123);
    (void)randnumber(0, 1); /* the first call seeds from time(); reseed after it, as the golden script did */
    srand(123);
    generateMatrix(&m, &n, &k, &init, &lo, &hi, w, h, NULL, &o);
    fwrite(w, sizeof(double), (size_t)m * k, f);
    fwrite(h, sizeof(double), (size_t)k * n, f);
    free(w);
    free(h);
  }
  /* the unsupported init and the missing-buffer path answer through errno without writing */
  {
    int k = 2;
    init_t init = nndsvd;
    double w[2000], h[80];
    errno = 0;
    generateMatrix(&m, &n, &k, &init, &lo, &hi, w, h, NULL, &o);
    if (errno != ENOSYS) return fail("generateMatrix nndsvd");
    errno = 0;
    init = ran;
    generateMatrix(&m, &n, &k, &init, &lo, &hi, NULL, h, NULL, &o);
    if (errno != EINVAL) return fail("generateMatrix NULL W");
  }
  fclose(f);
  printf("compat driver ok\n");
  return 0;
}
