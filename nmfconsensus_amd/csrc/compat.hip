// compat.hip -- the libnmf entry points of include/libnmf_compat.h, MI355X-native.
// nmf_mu's loop runs on the batched engine (engine.hip) with a batch of one restart; calculateNorm /
// calculateMaxchange are GPU reductions; the option helpers and the rand()-based init stay host C,
// exactly as the reference's (they share libc's global rand() state with the caller).
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <cstring>
#include <mutex>
#include <algorithm>
#include <vector>

#include "../../include/libnmf_compat.h"
#include "../../include/nmfc.h"
#include "nmfc_kernels.hpp"

namespace {
constexpr size_t NORM_BLOCKS = 4096;   // grid of the norm / max-change partial passes (>> 256 CUs)
}

extern "C" {

// setdefaultopts.c:38-52
void set_default_opts(options_t* opts) {
  opts->rep = 1;
  opts->init = ran;
  opts->min_init = 0;
  opts->max_init = 1;
  opts->w_out = "final_w.matrix";
  opts->h_out = "final_h.matrix";
  opts->TolX = 1.0E-04;
  opts->TolFun = 1.0E-04;
  opts->nndsvd_maxiter = -1;
  opts->nndsvd_blocksize = 64;
  opts->nndsvd_tol = 2E-16;
  opts->nndsvd_ncv = -1;
}

// checkarguments.c:50-78 -- same predicate, same errno and message
int checkArguments(const char* a, const int k, int iter, const char* w0, const char* h0, options_t* opts) {
  if (!a || k < 0 || iter < 0 || (w0 && w0[0] == '\0') || (h0 && h0[0] == '\0') || opts->rep < 0 ||
      opts->min_init < 0 || !opts->w_out || !opts->h_out || opts->TolX < 0 || opts->TolFun < 0) {
    errno = EDOM;
    perror("Error in arguments passed to nmfDriver.");
    return 1;
  }
  return 0;
}

// checkmatrices.c:43-81
int checkMatrices(const double* a, const double* w, const double* h, const int m, const int n, const int k) {
  long i;
  for (i = 0; i < (long)m * n && a[i] >= 0.; i++) {
  }
  if (i < (long)m * n) {
    printf("negative element in a[%ld]\n", i);
    return 1;
  }
  for (i = 0; i < (long)m * k && w[i] >= 0.; i++) {
  }
  if (i < (long)m * k) {
    printf("negative element in w[%ld] = %f\n", i, w[i]);
    return 1;
  }
  for (i = 0; i < (long)k * n && h[i] >= 0.; i++) {
  }
  if (i < (long)k * n) {
    printf("negative element in h[%ld]\n", i);
    return 1;
  }
  return 0;
}

// randnumber.c:27-35 -- libc rand(), time-seeded on first use like the reference
double randnumber(const int min, const int max) {
  static int initialised = 0;
  if (!initialised) {
    srand((unsigned)time(NULL));
    initialised = 1;
  }
  const int prod = (int)((unsigned)(max - min) * (unsigned)rand());
  return (double)min + ((double)prod / (double)(RAND_MAX));
}

// generatematrix.c:96-137 (ran); nndsvd (generatematrix.c:138-294) is out of scope -> ENOSYS.
// The reference returns WITHOUT filling W/H whenever errno is non-zero on entry (generatematrix.c:86-90 under
// ERROR_CHECKING, common.h:25: a stale errno from any earlier libc call is enough).  This entry point fills W/H
// regardless (the caller asked for an init); NMFC_GENERATE_ERRNO_COMPAT=1 restores the reference's early return.
void generateMatrix(const int* pm, const int* pn, const int* pk, init_t* pinit, const int* pmin, const int* pmax,
                    double* matrixW, double* matrixH, double* matrixA, options_t* opts) {
  (void)matrixA;
  (void)opts;
  const int m = *pm, n = *pn, k = *pk;
  if (errno) {
    const char* compat = getenv("NMFC_GENERATE_ERRNO_COMPAT");
    if (compat && atoi(compat) != 0) {
      perror("Failed to allocate memory in generateMatrix");
      return;
    }
  }
  if (!matrixW || !matrixH) {
    // the reference mallocs a buffer the caller never sees (generatematrix.c:118-121)
    errno = EINVAL;
    perror("generateMatrix: W and H buffers must be provided");
    return;
  }
  if (*pinit == ran) {
    for (long i = 0; i < (long)m * k; ++i) matrixW[i] = randnumber(*pmin, *pmax);
    for (long i = 0; i < (long)k * n; ++i) matrixH[i] = randnumber(*pmin, *pmax);
  } else {
    errno = ENOSYS;
    perror("generateMatrix: nndsvd initialisation is not provided by this engine");
  }
}

// The engine behind nmf_mu is kept across calls with the same A (nmf.r calls nmf_mu once per restart on
// one data matrix, nmf.r:41-45; R passes a fresh copy each time, so A is matched by shape and content: a
// host copy of the cached A is compared byte for byte, one pass over A like the hash it replaces, and no
// collision can reuse a stale A).  Creating an engine uploads A and builds its two layouts, and its first run
// allocates the work buffers: on the gct shape that is several times the whole MU loop.  A failed run drops
// the cached engine.  NMFC_NMF_MU_CACHE=0 disables the cache; nmfc_nmf_mu_release() frees it (HBM + host copy).
namespace {
std::mutex g_mu_lock;
struct MuCache {
  nmfc_engine* e = nullptr;
  int m = 0, n = 0;
  std::vector<double>* a = nullptr;   // host copy of the cached A (no destructor: HIP may be torn down at exit)
} g_mu;

void mu_cache_drop() {   // g_mu_lock held
  nmfc_engine_destroy(g_mu.e);
  g_mu.e = nullptr;
  g_mu.m = g_mu.n = 0;
  delete g_mu.a;
  g_mu.a = nullptr;
}
}  // namespace

void nmfc_solo_release();   // solo.hip

void nmfc_nmf_mu_release(void) {
  {
    std::lock_guard<std::mutex> lock(g_mu_lock);
    mu_cache_drop();
  }
  nmfc_solo_release();
}

// nmf_mu.c:84-315 on the GPU engine
double nmf_mu(double* a, double* w0, double* h0, int* pm, int* pn, int* pk, int* maxiter, const double* pTolX,
              const double* pTolFun) {
  (void)pTolX;
  (void)pTolFun;   // read but unused, as in the reference (nmf_mu.c:92-93)
  const int m = *pm, n = *pn, k = *pk;
  if (*maxiter < 1) {
    printf("Exiting nmf_mu after %i\n", 1);
    return 0;
  }
  if (k < 1 || k > m || k > n) {   // checked before any device work (libnmf_compat.h)
    fprintf(stderr, "Error in nmf_mu: k=%d unsupported (need 1 <= k <= min(m, n))\n", k);
    return -1;
  }
  if (k < 2 || k > nmfc::KMAX) {   // ranks outside the MFMA engine's 2..16: the generic GPU path
    int iters = 0, early = 0;
    if (nmfc_mu_generic(a, m, n, k, *maxiter, NMFC_STOP_REF_COMPAT, w0, h0, &iters, &early) != 0) {
      fprintf(stderr, "Error in nmf_mu: %s\n", nmfc_last_error());
      return -1;
    }
    int printed = iters;
    if (early)
      *maxiter = iters;
    else
      printed = iters + 1;
    printf("Exiting nmf_mu after %i\n", printed);
    return 0;
  }
  // rank 2..4 on a gct-sized matrix: one workgroup runs the whole restart (csrc/solo.hip); NMFC_SOLO=0 disables.
  // Ranks 5..8 take the team below for ONE call (7.6 vs 11.5 us per iteration at k = 5 on the gct: sixteen CUs'
  // latency against one CU's); a batch runs them on k_solo8_mu, one CU per restart, which carries more restarts.
  const char* solo_env = getenv("NMFC_SOLO");
  if (k <= 4 && nmfc_mu_solo_fits(m, n, k) && !(solo_env && atoi(solo_env) == 0)) {
    int iters = 0, early = 0;
    if (nmfc_mu_solo(a, m, n, k, *maxiter, NMFC_STOP_REF_COMPAT, w0, h0, w0, h0, &iters, &early) != 0) {
      fprintf(stderr, "Error in nmf_mu: %s\n", nmfc_last_error());
      return -1;
    }
    int printed = iters;
    if (early)
      *maxiter = iters;
    else
      printed = iters + 1;
    printf("Exiting nmf_mu after %i\n", printed);
    return 0;
  }
  const char* cache_env = getenv("NMFC_NMF_MU_CACHE");
  const bool cache = !(cache_env && atoi(cache_env) == 0);
  std::unique_lock<std::mutex> lock(g_mu_lock, std::defer_lock);
  nmfc_engine* e = nullptr;
  if (cache) {
    lock.lock();
    const size_t len = (size_t)m * n;
    if (g_mu.e && g_mu.m == m && g_mu.n == n && memcmp(g_mu.a->data(), a, len * sizeof(double)) == 0) {
      e = g_mu.e;
    } else {
      mu_cache_drop();
      e = nmfc_engine_create(-1, a, m, n, 0);
      if (e) {
        g_mu.e = e;
        g_mu.m = m;
        g_mu.n = n;
        g_mu.a = new std::vector<double>(a, a + len);
      }
    }
  } else {
    e = nmfc_engine_create(-1, a, m, n, 0);
  }
  if (!e) {
    fprintf(stderr, "Error in nmf_mu: %s\n", nmfc_last_error());
    return -1;
  }
  int32_t iters = 0, early = 0;
  // small shapes (the bundled gct, expression sets up to 8192 genes x 64 samples): one team launch with a single
  // upload / download (nmfc_engine_mu1); any other shape: the batched engine with a batch of one restart
  const long m_pad = ((long)m + 127) / 128 * 128;
  const char* team_env = getenv("NMFC_SMALL_KERNEL");
  const char* small_env = getenv("NMFC_SMALL");
  const bool team = m_pad <= 8192 && n <= 64 && !(team_env && strcmp(team_env, "single") == 0) &&
                    !(small_env && atoi(small_env) == 0);
  int rc = -1;
  if (team) {
    // w0/h0 are written only on success; a team that could not meet (its workgroups not all resident, e.g.
    // many processes sharing the GPU, as BatchJobs njobs > 1 does) reports it instead of hanging, and the
    // restart then runs on the batched engine, whose launches never wait for each other
    // NMFC_TEAM_FAIL=1 (tests only) takes the fallback as if the team had failed
    const char* tf = getenv("NMFC_TEAM_FAIL");
    if (!(tf && atoi(tf) != 0))
      rc = nmfc_engine_mu1(e, k, *maxiter, NMFC_STOP_REF_COMPAT, w0, h0, w0, h0, &iters, &early);
  }
  if (rc != 0) {
    nmfc_sweep_opts o;
    nmfc_default_opts(&o);
    o.maxiter = *maxiter;
    o.stop_rule = NMFC_STOP_REF_COMPAT;
    o.check_every = 64;
    nmfc_result r = {};
    r.iters = &iters;
    r.stopped_early = &early;
    r.W = w0;
    r.H = h0;
    const int ks[1] = {k};
    rc = nmfc_engine_run(e, ks, 1, 1, &o, w0, h0, &r);
  }
  if (!cache)
    nmfc_engine_destroy(e);
  else if (rc != 0)
    mu_cache_drop();   // the engine may be in a broken state: never reuse it
  if (rc != 0) {
    fprintf(stderr, "Error in nmf_mu: %s\n", nmfc_last_error());
    return -1;
  }
  // nmf_mu.c:270 writes *maxiter only on the early exit; :296 prints the loop counter (cap + 1 when
  // the loop ran to the cap).
  int printed = iters;
  if (early)
    *maxiter = iters;
  else
    printed = iters + 1;
  printf("Exiting nmf_mu after %i\n", printed);
  return 0;
}

// calculatenorm.c:44-78 on device operands: d = a - w h and ||d||_F / sqrt(m n), one fused GPU pass +
// a host sum of the per-block partials in block order (deterministic).  ms_out: device time of the pass.
int nmfc_calculate_norm_dev(const double* da, const double* dw, const double* dh, double* dd, int m, int n, int k,
                            double* norm_out, double* ms_out, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!da || !dw || !dh || !dd || m <= 0 || n <= 0 || k <= 0 || !norm_out) return -1;
  // grid: gene blocks x column groups (>> 256 CUs of workgroups; fixed for (m, n): deterministic sum order)
  const int gx = (m + nmfc::NT - 1) / nmfc::NT;
  const int gy = std::max(1, std::min(n, (int)((NORM_BLOCKS + gx - 1) / gx)));
  const int blocks = gx * gy;
  std::vector<double> part(blocks);
  double* dp = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  int rc = -1;
  if (hipMallocAsync((void**)&dp, blocks * 8, st) != hipSuccess) goto done;   // stream-ordered: no device sync
  if (ms_out && (hipEventCreate(&ev[0]) != hipSuccess || hipEventCreate(&ev[1]) != hipSuccess)) goto done;
  if (ms_out) (void)hipEventRecord(ev[0], st);
  switch (k) {   // rank known at compile time up to KMAX (the engine's range); the generic pass above it
#define NMFC_NORM_K(KK)                                                                                        \
  case KK:                                                                                                    \
    hipLaunchKernelGGL(nmfc::k_norm_partial_k<KK>, dim3(gx, gy), dim3(nmfc::NT), 0, st, da, dw, dh, dd, m, n, dp); \
    break;
    NMFC_NORM_K(1) NMFC_NORM_K(2) NMFC_NORM_K(3) NMFC_NORM_K(4) NMFC_NORM_K(5) NMFC_NORM_K(6) NMFC_NORM_K(7)
    NMFC_NORM_K(8) NMFC_NORM_K(9) NMFC_NORM_K(10) NMFC_NORM_K(11) NMFC_NORM_K(12) NMFC_NORM_K(13)
    NMFC_NORM_K(14) NMFC_NORM_K(15) NMFC_NORM_K(16)
#undef NMFC_NORM_K
    default:
      hipLaunchKernelGGL(nmfc::k_norm_partial, dim3(gx, gy), dim3(nmfc::NT), 0, st, da, dw, dh, dd, m, n, k, dp);
  }
  if (hipGetLastError() != hipSuccess) goto done;
  if (ms_out) (void)hipEventRecord(ev[1], st);
  if (hipMemcpyAsync(part.data(), dp, blocks * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    goto done;
  {
    double ss = 0.0;
    for (int b = 0; b < blocks; ++b) ss += part[b];
    *norm_out = sqrt(ss) / sqrt((double)m * n);
  }
  if (ms_out) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, ev[0], ev[1]);
    *ms_out = ms;
  }
  rc = 0;
done:
  for (hipEvent_t x : ev)
    if (x) (void)hipEventDestroy(x);
  if (dp) {
    (void)hipFreeAsync(dp, st);
    (void)hipStreamSynchronize(st);
  }
  return rc;
}

// calculatemaxchange.c:42-71 on device operands: max|mat0 - mat| / (sqrteps + max|mat0|); mat0 -= mat
// (exact and order-free).
int nmfc_calculate_maxchange_dev(const double* dm, double* dm0, int m, int n, double sqrteps, double* out,
                                 double* ms_out, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!dm || !dm0 || m <= 0 || n <= 0 || !out) return -1;
  const size_t len = (size_t)m * n;
  const int blocks = (int)std::min<size_t>((len + nmfc::NT - 1) / nmfc::NT, NORM_BLOCKS);
  std::vector<double> part(2 * blocks);
  double* dp = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  int rc = -1;
  if (hipMallocAsync((void**)&dp, 2 * blocks * 8, st) != hipSuccess) goto done;
  if (ms_out && (hipEventCreate(&ev[0]) != hipSuccess || hipEventCreate(&ev[1]) != hipSuccess)) goto done;
  if (ms_out) (void)hipEventRecord(ev[0], st);
  hipLaunchKernelGGL(nmfc::k_maxchange_partial, dim3(blocks), dim3(nmfc::NT), 0, st, dm, dm0, (long)len, dp);
  if (hipGetLastError() != hipSuccess) goto done;
  if (ms_out) (void)hipEventRecord(ev[1], st);
  if (hipMemcpyAsync(part.data(), dp, 2 * blocks * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    goto done;
  {
    double mx0 = 0.0, mxd = 0.0;
    for (int b = 0; b < blocks; ++b) {
      mx0 = fmax(mx0, part[2 * b]);
      mxd = fmax(mxd, part[2 * b + 1]);
    }
    *out = mxd / (sqrteps + mx0);
  }
  if (ms_out) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, ev[0], ev[1]);
    *ms_out = ms;
  }
  rc = 0;
done:
  for (hipEvent_t x : ev)
    if (x) (void)hipEventDestroy(x);
  if (dp) {
    (void)hipFreeAsync(dp, st);
    (void)hipStreamSynchronize(st);
  }
  return rc;
}

// calculatenorm.c:44-78 -- host operands: upload, nmfc_calculate_norm_dev, download d.
double calculateNorm(double* a, double* w, double* h, double* d, int m, int n, int k) {
  const size_t la = (size_t)m * n, lw = (size_t)m * k, lh = (size_t)k * n;
  double *da = nullptr, *dw = nullptr, *dh = nullptr, *dd = nullptr;
  double result = NAN, v = 0.0;
  if (hipMalloc(&da, la * 8) || hipMalloc(&dw, lw * 8) || hipMalloc(&dh, lh * 8) || hipMalloc(&dd, la * 8)) goto done;
  if (hipMemcpy(da, a, la * 8, hipMemcpyHostToDevice) || hipMemcpy(dw, w, lw * 8, hipMemcpyHostToDevice) ||
      hipMemcpy(dh, h, lh * 8, hipMemcpyHostToDevice))
    goto done;
  if (nmfc_calculate_norm_dev(da, dw, dh, dd, m, n, k, &v, nullptr, nullptr) != 0) goto done;
  if (hipMemcpy(d, dd, la * 8, hipMemcpyDeviceToHost)) goto done;
  result = v;
done:
  if (std::isnan(result)) fprintf(stderr, "calculateNorm: device failure\n");
  (void)hipFree(da);
  (void)hipFree(dw);
  (void)hipFree(dh);
  (void)hipFree(dd);
  return result;
}

// calculatemaxchange.c:42-71 -- host operands: upload, nmfc_calculate_maxchange_dev, download mat0.
double calculateMaxchange(double* mat, double* mat0, int m, int n, const double sqrteps) {
  const size_t len = (size_t)m * n;
  double *dm = nullptr, *dm0 = nullptr;
  double result = NAN, v = 0.0;
  if (hipMalloc(&dm, len * 8) || hipMalloc(&dm0, len * 8)) goto done;
  if (hipMemcpy(dm, mat, len * 8, hipMemcpyHostToDevice) || hipMemcpy(dm0, mat0, len * 8, hipMemcpyHostToDevice))
    goto done;
  if (nmfc_calculate_maxchange_dev(dm, dm0, m, n, sqrteps, &v, nullptr, nullptr) != 0) goto done;
  if (hipMemcpy(mat0, dm0, len * 8, hipMemcpyDeviceToHost)) goto done;
  result = v;
done:
  if (std::isnan(result)) fprintf(stderr, "calculateMaxchange: device failure\n");
  (void)hipFree(dm);
  (void)hipFree(dm0);
  return result;
}

}  // extern "C"
