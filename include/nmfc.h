/*
 * include/nmfc.h -- batched MI355X restart-sweep engine (additive C ABI of nmfconsensus_amd/libnmf.so).
 *
 * One call replaces the reference's restart fan-out and consensus reduction:
 *   createJobArray / runNMFinJobs   nmf.r:53-70, 106-113  (k x restart job grid, per-job seeds)
 *   doNMF                           nmf.r:23-51           (per-job init + .C("nmf_mu"))
 *   nmf_mu loop + stop rule         libnmf/nmf_mu.c:167-293
 *   computeConsensusMatrixFromClusterings  nmf.r:121-144 (labels, connectivity counts, /R)
 *   cophenetic correlation          nmf.r:165-172         (nmfc_cophenetic)
 * Plain pointers and sizes only.  All matrices are column-major fp64 like libnmf.
 */
#ifndef NMFC_H
#define NMFC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Stop rules (DESIGN.md "Stop rules"). */
enum {
  NMFC_STOP_FIXED = 0,          /* run exactly maxiter iterations */
  NMFC_STOP_REF_COMPAT = 1,     /* nmf_mu.c:253-282 as the reference executes it (zero-padded h0) */
  NMFC_STOP_ARGMAX_STABLE = 2,  /* same counter, per-sample argmax class (the check's intent) */
  NMFC_STOP_TOLX = 3            /* libnmf's TolX/TolFun convergence test (nmf_als.c:304-349 pattern, applied
                                   to the MU update): on even iterations > 1 stop when
                                   max(calculateMaxchange(W), calculateMaxchange(H)) < TolX, or when
                                   TolFun >= 1 (dnorm <= TolFun * dnorm0 with dnorm0 == dnorm, :330/:345) */
};

/* Initialisation streams of the per-job W0/H0. */
enum {
  NMFC_INIT_LIBNMF = 0,         /* libnmf generateMatrix(ran): glibc rand() after srand(job seed)
                                   (generatematrix.c:94-100, randnumber.c:27-35; the north-star stream) */
  NMFC_INIT_R_RUNIF = 1         /* nmf.r:37-38: set.seed(job seed); W <- runif(m*k); H <- runif(k*n)
                                   (R's Mersenne-Twister; BatchJobs job seed = seed + job_id - 1) */
};

/* Label rules for the consensus (nmf.r:128). */
enum {
  NMFC_LABEL_ARGMAX = 0,        /* row of the column maximum (nmf.r:127 comment, BROAD intent) */
  NMFC_LABEL_R_ORDER = 1        /* apply(H,2,order)[1,] as written at nmf.r:128: the column minimum */
};

typedef struct nmfc_sweep_opts {
  int maxiter;        /* nmf.r maxniter (cap; default 10000) */
  int stop_rule;      /* NMFC_STOP_* */
  int label_rule;     /* NMFC_LABEL_* */
  uint32_t seed;      /* registry seed: job seed = seed + job_id - 1 (job_id 1-based, expand.grid order) */
  int min_init;       /* generateMatrix range (options_t.min_init / max_init, default 0 / 1) */
  int max_init;
  int job_begin;      /* shard [job_begin, job_end) of the 0-based job list; job_end < 0 => all jobs */
  int job_end;
  int check_every;    /* host polls the stopped-restart count every this many iterations (default 4) */
  int verbose;        /* 0 quiet; 1 per-sweep summary on stderr */
  double TolX;        /* NMFC_STOP_TOLX threshold (options_t.TolX, default 1e-4, setdefaultopts.c) */
  double TolFun;      /* NMFC_STOP_TOLX TolFun (default 1e-4) */
  int init_stream;    /* NMFC_INIT_* (default NMFC_INIT_LIBNMF; min_init/max_init apply to LIBNMF only) */
} nmfc_sweep_opts;

/* Outputs.  Every pointer may be NULL.  Host memory unless *_on_device is set.
 * Jobs are indexed 0..njobs-1 in expand.grid order (k fastest): job j has k = ks[j % nk] and restart
 * r = j / nk + 1; per-job arrays are indexed by (j - job_begin). */
typedef struct nmfc_result {
  int32_t* counts;          /* nk x n x n integer connectivity counts of this shard's jobs */
  int counts_on_device;     /* counts is a device pointer (e.g. a torch tensor for an RCCL all-reduce) */
  double* consensus;        /* nk x n x n  counts / R  (only meaningful for a full, unsharded run) */
  int32_t* labels;          /* njobs_shard x n, 1-based */
  int32_t* iters;           /* njobs_shard: iterations run */
  int32_t* stopped_early;   /* njobs_shard: 1 if the stop rule fired (nmf_mu.c:270 writes *maxiter), else 0 */
  double* W;                /* sum over shard jobs of m*k, job-major, each m x k column-major */
  double* H;                /* sum over shard jobs of k*n, job-major, each k x n column-major */
  /* filled by the engine: */
  double seconds_total;     /* wall time of the run inside the engine */
  double seconds_iterate;   /* part spent in the iteration loop */
  long long restart_iterations; /* sum of iterations over the shard's restarts */
  int max_iter_run;         /* largest iteration count */
} nmfc_result;

typedef struct nmfc_engine nmfc_engine;

/* Creates an engine on HIP device `device` (-1: current device) with data matrix A (m x n, ld m).
 * a_on_device != 0: A is a device pointer (copied device-to-device into the engine's layouts). */
nmfc_engine* nmfc_engine_create(int device, const double* A, int m, int n, int a_on_device);
void nmfc_engine_destroy(nmfc_engine* e);
/* The HIP device ordinal the engine was created on (resolved at creation when device was -1); -1 for NULL. */
int nmfc_engine_device(const nmfc_engine* e);

/* The calling thread's current HIP device ordinal (what device -1 resolves to), or -1 on failure. */
int nmfc_current_device(void);

void nmfc_default_opts(nmfc_sweep_opts* o);

/* Runs the k-sweep: for every job of the shard, init (generateMatrix(ran) stream with the job seed,
 * or the caller's W_init/H_init when given), MU iterations under the stop rule, labels, counts.
 * W_init / H_init (optional): job-major initial factors for the shard, layouts as in nmfc_result.
 * Returns 0 on success; nonzero with nmfc_last_error() set otherwise. */
int nmfc_engine_run(nmfc_engine* e, const int* ks, int nk, int R, const nmfc_sweep_opts* opts,
                    const double* W_init, const double* H_init, nmfc_result* out);

/* Convenience: create, run, destroy. */
/* One restart of nmf_mu (nmf_mu.c:84-315) on the small-shape team kernel (m rounded up to 128 <= 8192, n <= 64,
 * k <= 16), with one upload, one launch and one download: the per-call path of the nmf_mu drop-in (nmf.r:41-45).
 * W0 (m x k) and H0 (k x n) column-major as nmf_mu takes them; W_out/H_out may alias them.  *iters = the
 * iterations run, *early = 1 when the stop rule (not maxiter) ended the loop.  stop_rule: FIXED, REF_COMPAT or
 * ARGMAX_STABLE.  Returns 0, or -1 (nmfc_last_error) also for a shape outside the team range. */
int nmfc_engine_mu1(nmfc_engine* e, int k, int maxiter, int stop_rule, const double* W0, const double* H0, double* W_out,
                    double* H_out, int* iters, int* early);
/* One restart of nmf_mu for any rank 1 <= k <= min(m, n) on the generic GPU path (ranks the MFMA engine does not
 * take, k > 16 or k = 1): the six products of nmf_mu.c:174-202 as plain fp64 contractions, the rules and the stop
 * check as small kernels; A is kept on the device across calls with the same A (compared byte for byte).  Same
 * argument meaning as nmfc_engine_mu1 (W m x k, H k x n column-major, updated in place). */
int nmfc_mu_generic(const double* A, int m, int n, int k, int maxiter, int stop_rule, double* W, double* H, int* iters,
                    int* early);
/* One restart of nmf_mu of rank 2 <= k <= 4 on a small matrix (k <= m <= 1024, k <= n <= 40) on ONE workgroup:
 * the whole MU loop and stop rule in one launch, A resident in that CU's registers (and LDS) (csrc/solo.hip).
 * The drop-in's path for the bundled gct at k = 2..4.  W0/H0 in, W/H out (column-major, may alias),
 * *iters / *early as nmfc_engine_mu1; A cached on the device across calls (compared byte for byte).  Returns 0, or
 * -1 (nmfc_last_error) for a shape outside the range (nmfc_mu_solo_fits says which shapes fit). */
int nmfc_mu_solo_fits(int m, int n, int k);
int nmfc_mu_solo(const double* A, int m, int n, int k, int maxiter, int stop_rule, const double* W0, const double* H0,
                 double* W, double* H, int* iters, int* early);
int nmfc_sweep(const double* A, int m, int n, const int* ks, int nk, int R, const nmfc_sweep_opts* opts,
               nmfc_result* out);

/* computeConsensusMatrixFromClusterings (nmf.r:121-144) on the GPU for R results of one rank k:
 * Hs holds R consecutive k x n column-major H matrices (host).  labels (R x n, 1-based), counts (n x n
 * int) and consensus (n x n, counts / R) are host outputs; each may be NULL. */
int nmfc_consensus(const double* Hs, int k, int n, int R, int label_rule, int32_t* labels, int32_t* counts,
                   double* consensus);

/* Cophenetic correlation of one consensus matrix (nmf.r:165-172): average-linkage hclust on
 * d = 1 - C, cophenetic distances, Pearson correlation over the n(n-1)/2 pairs (unrounded; R
 * applies signif(., 4) afterwards).  order_out (n, 1-based, may be NULL) receives the dendrogram
 * leaf order (HC$order); merge_out (2*(n-1), may be NULL) R-style merge matrix; height_out (n-1). */
double nmfc_cophenetic(const double* C, int n, int32_t* order_out, int32_t* merge_out, double* height_out);

/* nmfc_cophenetic for nk consensus matrices (nk x n x n, each column-major) on up to nthreads host threads
 * (<= 0: all hardware threads); rho_out[nk]; order_out (nk x n), merge_out (nk x 2(n-1)), height_out
 * (nk x (n-1)) may be NULL.  Returns 0, or -1 on bad arguments. */
int nmfc_cophenetic_batch(const double* C, int nk, int n, int nthreads, double* rho_out, int32_t* order_out,
                          int32_t* merge_out, double* height_out);

/* cutree(HC, k) membership (nmf.r:177) from a merge matrix produced by nmfc_cophenetic. 1-based. */
int nmfc_cutree(const int32_t* merge, int n, int k, int32_t* membership_out);

/* ---------------------------------------------------------------------------------------------
 * Brunet KL-divergence MU restarts (BASELINE.json configs[4]).  The per-restart
 * algorithm is the BROAD nmfconsensus script's NMF.div (Brunet et al. 2004), which the reference only
 * names (commented-out call, test_nmf.r:29); restated in oracle/brunet_oracle.c, parity vs the
 * reference unpinned.  Job order follows nmfconsensus: for k in ks, for restart i in 1..R, with
 * set.seed(seed + i) then W <- runif(m*k), H <- runif(k*n) (R's Mersenne-Twister, bit-exact).
 * Per-job output arrays are indexed (k index) * (restart_end - restart_begin) + (i - 1 - restart_begin);
 * W/H outputs are job-major in that order (W m x k, H k x n, column-major).  counts/consensus as for
 * nmfc_engine_run (membership = order(H[,j], decreasing=TRUE)[1], i.e. the first row of the maximum).
 * --------------------------------------------------------------------------------------------- */
typedef struct nmfc_brunet_opts {
  int maxiter;        /* NMF.div maxniter (default 2000) */
  int stopconv;       /* consecutive unchanged membership checks that stop a restart (default 40) */
  int stopfreq;       /* iterations between membership checks (default 10) */
  uint32_t seed;      /* nmfconsensus rseed: restart i (1-based) uses set.seed(seed + i) (default 123456789) */
  int restart_begin;  /* shard [restart_begin, restart_end) of the restarts 0..R-1, for every k; end < 0 => R */
  int restart_end;
  int verbose;
  int lanes;          /* k batches run concurrently, each on its own HIP stream (0 = default 4, max 4) */
} nmfc_brunet_opts;

typedef struct nmfc_brunet nmfc_brunet;

void nmfc_brunet_default_opts(nmfc_brunet_opts* o);
/* A: m x n column-major, every entry finite, >= 0 and <= 2^64 (else NULL with nmfc_last_error set): the domain in
 * which the kernels' batched reciprocals stay normal (csrc/brunet.hip recip_batch). */
nmfc_brunet* nmfc_brunet_create(int device, const double* A, int m, int n, int a_on_device);
void nmfc_brunet_destroy(nmfc_brunet* e);
int nmfc_brunet_device(const nmfc_brunet* e);   /* as nmfc_engine_device */
/* W_init/H_init (optional, host): every job of the shard in output order, entries in [2^-60, 2^60].
 * Returns 0 or -1 (nmfc_last_error). */
int nmfc_brunet_run(nmfc_brunet* e, const int* ks, int nk, int R, const nmfc_brunet_opts* opts, const double* W_init,
                    const double* H_init, nmfc_result* out);
void nmfc_brunet_set_timing(nmfc_brunet* e, int enable);
/* kernel ids 0 = H-side quotient product (k_br_hnum), 1 = H update + check (k_br_hupd), 2 = W side
 * (k_br_wupd); returns launches, fills accumulated event ms and algorithmic flop per launch. */
long long nmfc_brunet_kernel_time(nmfc_brunet* e, int kernel_id, double* ms_out, double* flops_per_launch);

/* calculateNorm (calculatenorm.c:44-78) and calculateMaxchange (calculatemaxchange.c:42-71) on
 * DEVICE-resident column-major operands (e.g. torch tensors) on the current HIP device: d = a - w h and
 * *norm_out = ||d||_F / sqrt(m n); *out = max|mat0 - mat| / (sqrteps + max|mat0|) with mat0 -= mat.
 * stream: the hipStream_t (as void*) the operands were produced on; the pass and its partials buffer are
 * ordered on it (NULL: the null stream), and the call returns after it has finished.
 * ms_out (may be NULL) receives the device time of the reduction pass.  Return 0, or -1 on failure. */
int nmfc_calculate_norm_dev(const double* a, const double* w, const double* h, double* d, int m, int n, int k,
                            double* norm_out, double* ms_out, void* stream);
int nmfc_calculate_maxchange_dev(const double* mat, double* mat0, int m, int n, double sqrteps, double* out,
                                 double* ms_out, void* stream);

/* Frees the engine that nmf_mu (libnmf_compat.h) keeps across calls with the same A (its HBM and host copy). */
void nmfc_nmf_mu_release(void);

/* Diagnostics. */
const char* nmfc_last_error(void);

/* The compile-time tuning switches this library was built with, "NAME=value;..." as the preprocessor saw them in the
 * MU engine's / the Brunet kernels' translation unit (csrc/nmfc_tuning.hpp lists each with its product default; the
 * CPU suite checks the product build against those defaults). */
const char* nmfc_build_tuning(void);
const char* nmfc_build_tuning_brunet(void);
const char* nmfc_version(void);
/* Per-kernel device time (ms) accumulated over the last run, measured with HIP events on the
 * engine's stream: kernel ids 0 = wta (W^T A + W^T W, MFMA), 1 = hupdate (H update + stop check),
 * 2 = ahtw (A h^T MFMA + W update), 3 = init, 4 = other (repack moves, TolX W check), 5 = labels,
 * 6 = connectivity counts, 7 = small-shape persistent MU kernel (m_pad <= 1024, n <= 64: the whole
 * loop in one launch).  Returns the number of launches of that kernel. */
long long nmfc_engine_kernel_time(nmfc_engine* e, int kernel_id, double* ms_out);
/* enable = 0: no event timing; enable = S >= 1: HIP events around every launch of every S-th MU
 * iteration (and every other launch), so kernel_time returns the TIMED launches and their summed ms
 * (a uniform sample of the run; used by bench.py's roofline leg).  Flop/byte figures are per launch
 * over all launches. */
void nmfc_engine_set_timing(nmfc_engine* e, int enable);
/* Algorithmic flop per launch of the dominant kernel in the last run, for the roofline report. */
double nmfc_engine_kernel_flops(nmfc_engine* e, int kernel_id);
/* HBM bytes per launch in the last run: returns the bytes the kernel's design moves (operands once plus
 * split-K / Gram partials); *algo_bytes_out (may be NULL) receives the algorithmic bytes (each operand
 * once; the H update uses SURVEY 8(d)'s 32 n k per restart-iteration). */
double nmfc_engine_kernel_bytes(nmfc_engine* e, int kernel_id, double* algo_bytes_out);

#ifdef __cplusplus
}
#endif
#endif
