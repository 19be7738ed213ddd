/*
 * include/libnmf_compat.h -- the drop-in boundary: the libnmf entry points that the reference's
 * R driver binds (nmf.r:4,41-45 `dyn.load("libnmf.so")` + `.C("nmf_mu", ...)`), re-implemented
 * MI355X-native in nmfconsensus_amd/libnmf.so (soname libnmf.so).  Signatures, argument meaning,
 * ownership and error behaviour follow the reference exactly; the header cites the line each
 * declaration replaces.  Types keep the reference layout (libnmf/include/common.h:61-105).
 */
#ifndef NMFC_LIBNMF_COMPAT_H
#define NMFC_LIBNMF_COMPAT_H

#ifdef __cplusplus
extern "C" {
#endif

/* common.h:61-64 */
typedef struct idx_double {
  double val;
  int idx;
} idx_double;

/* common.h:78 */
typedef enum alg_t { mu, als, neals, alspg, pg } alg_t;

/* common.h:85 */
typedef enum init_t { ran, nndsvd } init_t;

/* common.h:92-105 */
typedef struct options_t {
  int rep;
  init_t init;
  int min_init;
  int max_init;
  const char* w_out;
  const char* h_out;
  double TolX;
  double TolFun;
  int nndsvd_maxiter;
  int nndsvd_blocksize;
  double nndsvd_tol;
  int nndsvd_ncv;
} options_t;

/*
 * nmf_mu -- replaces libnmf/nmf_mu.c:84-85 (header libnmf/include/nmf_mu.h:55-56).
 * a (m x n, ld m) is read only; w0 (m x k) / h0 (k x n) hold the initial factors on entry and the
 * final factors on exit -- ALWAYS, also for odd iteration counts (the reference leaves them there
 * only after an even count, nmf_mu.c:241-242).  *maxiter: in = cap, out = iteration of the early
 * exit (nmf_mu.c:270), unchanged when the cap is reached.  TolX/TolFun are read but unused, as in
 * the reference (nmf_mu.c:92-93, convergence code commented out at :220-237).  The iteration loop
 * runs on the GPU (HIP, gfx950).  Prints "Exiting nmf_mu after <iter>\n" like nmf_mu.c:296.
 * The stop rule is the reference's class-stability check (nmf_mu.c:253-282) in its defined
 * REF_COMPAT form.  Returns 0, or -1 on allocation / device failure (nmf_mu.c:138-151).
 * Ranks: 1 <= k <= min(m, n).  Routing, a function of (m, n, k) only (so a restart gives the same bits on every call):
 *   solo    k = 2..4 on gct-sized matrices (nmfc_mu_solo_fits: m <= 1024, n <= 40): ONE workgroup runs the whole
 *           restart, A resident in its register file (csrc/solo.hip, k_solo_mu; ranks 5..8 have a one-workgroup
 *           kernel too, k_solo8_mu, which batches use, but one call runs faster on a team);
 *   team    other k = 2..16 with m_pad = 128-rounded m <= 8192, n <= 64: a team of m_pad / 64 workgroups
 *           (k_team_mu, one launch with one upload / download);
 *   engine  other k = 2..16: the batched MFMA engine with a batch of one;
 *   generic any other k: plain fp64 products, one thread per output (nmfc_mu_generic, csrc/generic.hip).
 * A team that cannot assemble (its workgroups not all resident, e.g. while other processes hold the GPU's CUs, as
 * BatchJobs njobs > 1 runs it) reports so instead of waiting, and the restart runs on the engine; the solo kernel is
 * one workgroup and needs no such fallback.  k outside 1..min(m, n) prints
 * "Error in nmf_mu: k=<k> unsupported (need 1 <= k <= min(m, n))" to stderr before any device work, leaves
 * w0/h0 untouched and returns -1.
 */
double nmf_mu(double* a, double* w0, double* h0, int* pm, int* pn, int* pk, int* maxiter,
              const double* pTolX, const double* pTolFun);

/* set_default_opts -- replaces libnmf/setdefaultopts.c:38-52 */
void set_default_opts(options_t* opts);

/* checkArguments -- replaces libnmf/checkarguments.c:50-78 (returns 1 and sets errno=EDOM) */
int checkArguments(const char* a, const int k, int iter, const char* w0, const char* h0, options_t* opts);

/* checkMatrices -- replaces libnmf/checkmatrices.c:43-81 (returns 1 on a negative element) */
int checkMatrices(const double* a, const double* w, const double* h, const int m, const int n, const int k);

/* randnumber -- replaces libnmf/randnumber.c:27-35: min + ((max-min)*rand())/(double)RAND_MAX
 * drawn from libc rand(), seeded with srand(time(NULL)) on first use, like the reference. */
double randnumber(const int min, const int max);

/* generateMatrix -- replaces libnmf/generatematrix.c:59 (init == ran; generatematrix.c:131-137).
 * W (m*k) then H (k*n) from randnumber().  init == nndsvd is out of scope: W/H are left untouched
 * and errno is set to ENOSYS. */
void generateMatrix(const int* pm, const int* pn, const int* pk, init_t* pinit, const int* pmin, const int* pmax,
                    double* matrixW, double* matrixH, double* matrixA, options_t* opts);

/* calculateNorm -- replaces libnmf/calculatenorm.c:44-78: d = a - w*h; returns ||d||_F / sqrt(m*n).
 * Computed on the GPU (fused: d is produced and reduced in one pass). */
double calculateNorm(double* a, double* w, double* h, double* d, int m, int n, int k);

/* calculateMaxchange -- replaces libnmf/calculatemaxchange.c:42-71:
 * returns max|mat0 - mat| / (sqrteps + max|mat0|); side effect mat0 -= mat.  GPU reduction. */
double calculateMaxchange(double* mat, double* mat0, int m, int n, const double sqrteps);

#ifdef __cplusplus
}
#endif
#endif
