/* r_nmfc.c -- the R bindings of the batched engine (INTEGRATION.md sections 2 and 6), as a maintainer adds them next
 * to nmf.r:  R CMD SHLIB r_nmfc.c -L<lib dir> -lnmf   (or `make -C examples r_nmfc.so`, which build() runs).
 *
 * R's .C passes every argument as a pointer to R's own storage: integer vectors as int*, double vectors as double*;
 * output vectors are allocated by the caller (integer(nk*n*n), double(nk*n*n), ...) and filled in place.  No R
 * headers are needed.  tests/test_gpu_r_binding.py drives both entries through ctypes with exactly that convention.
 *
 *   r_nmfc_sweep   replaces runNMFinJobs' restart fan-out (nmf.r:106-119: createJobArray nmf.r:53-70, doNMF
 *                  nmf.r:23-51, BatchJobs submit/wait) and computeConsensusMatrixFromClusterings (nmf.r:121-144)
 *   r_nmfc_brunet  replaces the BROAD nmfconsensus() per-k loop over NMF.div + connect.matrix (test_nmf.r:29)
 */
#include <stdint.h>

#include "nmfc.h"

/* A: m x n column-major (as.double(A)); ks[nk]; R = num.clusterings; seed: the registry seed (job seed = seed +
 * job_id - 1); label_rule: 0 argmax (intent), 1 order()[1] as nmf.r:128; init_stream: 0 libnmf generateMatrix(ran),
 * 1 nmf.r:37-38's runif.  Outputs: counts / consensus nk x n x n, labels (nk R) x n (1-based, job-major), iters
 * nk R (expand.grid job order, k fastest); rc 0 on success. */
void r_nmfc_sweep(double* A, int* m, int* n, int* ks, int* nk, int* R, int* maxiter, int* seed, int* label_rule,
                  int* init_stream, int32_t* counts, double* consensus, int32_t* labels, int32_t* iters, int* rc) {
  nmfc_sweep_opts o;
  nmfc_result r = {0};
  nmfc_default_opts(&o);
  o.maxiter = *maxiter;
  o.seed = (uint32_t)*seed;
  o.label_rule = *label_rule;
  o.init_stream = *init_stream;
  r.counts = counts;
  r.consensus = consensus;
  r.labels = labels;
  r.iters = iters;
  *rc = nmfc_sweep(A, *m, *n, ks, *nk, *R, &o, &r);
}

/* Brunet KL-divergence MU sweep (GenePattern NMF.div): restart i of every k from set.seed(rseed + i) + runif;
 * stopconv / stopfreq as the script; outputs counts / consensus nk x n x n, iters nk R (k-major: the R restarts of
 * ks[0], then of ks[1], ...); rc 0 on success. */
void r_nmfc_brunet(double* A, int* m, int* n, int* ks, int* nk, int* R, int* maxiter, int* rseed, int* stopconv,
                   int* stopfreq, int32_t* counts, double* consensus, int32_t* iters, int* rc) {
  nmfc_brunet_opts o;
  nmfc_result r = {0};
  nmfc_brunet* e;
  nmfc_brunet_default_opts(&o);
  o.maxiter = *maxiter;
  o.seed = (uint32_t)*rseed;
  o.stopconv = *stopconv;
  o.stopfreq = *stopfreq;
  r.counts = counts;
  r.consensus = consensus;
  r.iters = iters;
  e = nmfc_brunet_create(-1, A, *m, *n, 0);
  *rc = e ? nmfc_brunet_run(e, ks, *nk, *R, &o, 0, 0, &r) : -1;
  nmfc_brunet_destroy(e);
}
