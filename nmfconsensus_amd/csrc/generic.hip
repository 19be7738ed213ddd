// generic.hip -- nmf_mu for ranks above the batched engine's limit (k > 16; the reference's nmf_mu takes any k,
// nmf_mu.c:84-85).  One restart per call, on the GPU: the six products of nmf_mu.c:174-202 as plain fp64
// contractions (one thread per output element, a sequential fma chain over K: deterministic), the two
// multiplicative rules (nmf_mu.c:184-191, 209-216) and the stability check (nmf_mu.c:253-282) as small kernels.
// Layouts are the reference's: A m x n, W m x k, H k x n, all column-major.  A rare path (consensus clustering
// sweeps k = 2..10 or so); the fast paths are the team kernel and the batched engine (engine.hip).
// Cost: W^T A runs k n threads, each a serial chain over all m genes, and an iteration is 9 dependent launches, so on a
// large matrix (e.g. 60000 x 2000 at k = 20: 40000 threads x 60000 dependent fmas) one iteration takes on the order of
// milliseconds -- correct and deterministic, not fast.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/nmfc.h"
#include "nmfc_kernels.hpp"

void nmfc_set_error(const char* msg);

namespace {

constexpr int GB = 256;

// C(r, c) = sum_{t < K} P(t, r) Q(t, c); element (t, r) of P at P[t * pt + r * pr], (t, c) of Q at Q[t * qt + c * qc],
// C(r, c) at C[r * cr + c * cc].  One thread per output, t in order.
__global__ __launch_bounds__(GB) void k_gen_prod(int M, int N, int K, const double* __restrict__ P, long pt, long pr,
                                                 const double* __restrict__ Q, long qt, long qc, double* __restrict__ C,
                                                 long cr, long cc) {
  const long x = (long)blockIdx.x * GB + threadIdx.x;
  if (x >= (long)M * N) return;
  const long r = x % M, c = x / M;
  const double* p = P + r * pr;
  const double* q = Q + c * qc;
  double s = 0.0;
  for (int t = 0; t < K; ++t) s = fma(p[t * pt], q[t * qt], s);
  C[r * cr + c * cc] = s;
}

// x = mu_rule(x, num, den) elementwise (nmf_mu.c:184-191 / 209-216), unless the restart has stopped
__global__ __launch_bounds__(GB) void k_gen_rule(long len, double* __restrict__ x, const double* __restrict__ num,
                                                 const double* __restrict__ den, const int* __restrict__ state) {
  if (state[0]) return;
  const long i = (long)blockIdx.x * GB + threadIdx.x;
  if (i < len) x[i] = nmfc::mu_rule(x[i], num[i], den[i]);
}

// state: [0] stopped, [1] stop iteration, [2] reason (1 stable, 2 maxiter), [3] unchanged checks; cls[n] classes.
// REF_COMPAT: window i < min(k, n) of the flat k x n buffer, class = last jj in [1, k) with h[i n + jj] > h[i n + jj - 1]
// (windows i >= k would read past the buffer, nmf_mu.c:259: the zero padding keeps them at class 0).
__global__ __launch_bounds__(GB) void k_gen_check(int iter, int maxiter, int stop_rule, int k, int n,
                                                  const double* __restrict__ H, int* __restrict__ cls,
                                                  int* __restrict__ state) {
  __shared__ int changed;
  if (state[0]) return;
  if (threadIdx.x == 0) changed = 0;
  __syncthreads();
  const bool check = stop_rule != nmfc::STOP_FIXED && iter > 1 && (iter % 2 == 0);
  if (check) {
    if (stop_rule == nmfc::STOP_REF_COMPAT) {
      for (int i = threadIdx.x; i < k && i < n; i += GB) {
        int c = 0;
        for (int jj = 1; jj < k; ++jj)
          if (H[(long)i * n + jj] > H[(long)i * n + jj - 1]) c = jj;
        if (cls[i] != c) {
          cls[i] = c;
          changed = 1;
        }
      }
    } else if (stop_rule == nmfc::STOP_ARGMAX_STABLE) {
      for (int j = threadIdx.x; j < n; j += GB) {
        int best = 0;
        double bv = H[(long)j * k];
        for (int a = 1; a < k; ++a)
          if (H[(long)j * k + a] > bv) {
            bv = H[(long)j * k + a];
            best = a;
          }
        if (cls[j] != best) {
          cls[j] = best;
          changed = 1;
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int reason = 0;
    if (check) {
      if (!changed) {
        if (++state[3] >= 200) reason = 1;   // nmf_mu.c:269-271
      } else {
        state[3] = 0;
      }
    }
    if (!reason && iter >= maxiter) reason = 2;
    if (reason) {
      state[0] = 1;
      state[1] = iter;
      state[2] = reason;
    }
  }
}

struct GenCache {   // device copy of the last A (compared byte for byte) and work buffers
  std::vector<double> a;
  int m = 0, n = 0;
  double* dA = nullptr;
  double* work = nullptr;
  size_t work_bytes = 0;
  int* state = nullptr;
  int* cls = nullptr;   // the stability check's classes (n of them)
  int cls_n = 0;
  hipStream_t st = nullptr;
  int dev = -1;         // the HIP device every resource above lives on
};
std::mutex g_lock;
GenCache g;

void cache_drop() {   // g_lock held
  if (g.st) (void)hipStreamSynchronize(g.st);
  if (g.dA) (void)hipFree(g.dA);
  if (g.work) (void)hipFree(g.work);
  if (g.state) (void)hipFree(g.state);
  if (g.cls) (void)hipFree(g.cls);
  if (g.st) (void)hipStreamDestroy(g.st);
  g.a.clear();
  g.a.shrink_to_fit();
  g.dA = g.work = nullptr;
  g.state = g.cls = nullptr;
  g.st = nullptr;
  g.work_bytes = 0;
  g.cls_n = 0;
  g.m = g.n = 0;
  g.dev = -1;
}

int mu_generic_call(const double* A, int m, int n, int k, int maxiter, int stop_rule, double* W, double* H, int* iters,
                    int* early);

int fail(const char* what, hipError_t e) {
  char buf[256];
  snprintf(buf, sizeof buf, "nmfc_mu_generic: %s: %s", what, hipGetErrorString(e));
  nmfc_set_error(buf);
  return -1;
}

}  // namespace

#define GCHECK(x)                          \
  do {                                     \
    hipError_t e_ = (x);                   \
    if (e_ != hipSuccess) return fail(#x, e_); \
  } while (0)

extern "C" int nmfc_mu_generic(const double* A, int m, int n, int k, int maxiter, int stop_rule, double* W, double* H,
                               int* iters, int* early) {
  if (!A || !W || !H || m < 1 || n < 1 || k < 1 || k > m || k > n || maxiter < 0 ||
      (stop_rule != NMFC_STOP_FIXED && stop_rule != NMFC_STOP_REF_COMPAT && stop_rule != NMFC_STOP_ARGMAX_STABLE)) {
    nmfc_set_error("nmfc_mu_generic: bad arguments");
    return -1;
  }
  std::lock_guard<std::mutex> lock(g_lock);
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return fail("hipGetDevice", hipErrorInvalidDevice);
  if (g.dev >= 0 && g.dev != dev) cache_drop();
  const int rc = mu_generic_call(A, m, n, k, maxiter, stop_rule, W, H, iters, early);
  // a failed call may leave a half-done upload behind: nothing of it is reused; NMFC_NMF_MU_CACHE=0 keeps nothing
  const char* env = getenv("NMFC_NMF_MU_CACHE");
  if (rc != 0 || (env && atoi(env) == 0))
    cache_drop();
  else
    g.dev = dev;
  return rc;
}

namespace {
int mu_generic_call(const double* A, int m, int n, int k, int maxiter, int stop_rule, double* W, double* H, int* iters,
                    int* early) {
  const size_t la = (size_t)m * n;
  if (!g.st) GCHECK(hipStreamCreateWithFlags(&g.st, hipStreamNonBlocking));
  if (!(g.dA && g.m == m && g.n == n && memcmp(g.a.data(), A, la * sizeof(double)) == 0)) {
    if (g.dA) (void)hipFree(g.dA);
    g.dA = nullptr;
    g.a.assign(A, A + la);
    g.m = m;
    g.n = n;
    GCHECK(hipMalloc(&g.dA, la * sizeof(double)));
    GCHECK(hipMemcpyAsync(g.dA, A, la * sizeof(double), hipMemcpyHostToDevice, g.st));
  }
  // work: W, H, numerh / hden (k x n), wtw / hht (k x k), numerw / wden (m x k)
  const size_t lw = (size_t)m * k, lh = (size_t)k * n, lk = (size_t)k * k;
  const size_t need = sizeof(double) * (3 * lw + 3 * lh + 2 * lk);
  if (g.work_bytes < need) {
    if (g.work) (void)hipFree(g.work);
    g.work = nullptr;
    g.work_bytes = 0;
    GCHECK(hipMalloc(&g.work, need));
    g.work_bytes = need;
  }
  if (!g.state) GCHECK(hipMalloc(&g.state, sizeof(int) * 8));
  double* dW = g.work;
  double* dH = dW + lw;
  double* numw = dH + lh;
  double* denw = numw + lw;
  double* numh = denw + lw;
  double* denh = numh + lh;
  double* wtw = denh + lh;
  double* hht = wtw + lk;
  if (g.cls_n < n) {
    if (g.cls) (void)hipFree(g.cls);
    g.cls = nullptr;
    g.cls_n = 0;
    GCHECK(hipMalloc(&g.cls, sizeof(int) * (size_t)n));
    g.cls_n = n;
  }
  int* cls = g.cls;
  GCHECK(hipMemsetAsync(cls, 0, sizeof(int) * (size_t)n, g.st));   // nmf_mu.c:132
  GCHECK(hipMemsetAsync(g.state, 0, sizeof(int) * 8, g.st));
  GCHECK(hipMemcpyAsync(dW, W, lw * sizeof(double), hipMemcpyHostToDevice, g.st));
  GCHECK(hipMemcpyAsync(dH, H, lh * sizeof(double), hipMemcpyHostToDevice, g.st));
  auto grid = [](long cnt) { return dim3((unsigned)((cnt + GB - 1) / GB)); };
  const double* dA = g.dA;
  int hstate[4] = {0, 0, 0, 0};
  int it = 0;
  for (; it < maxiter;) {
    const int chunk = std::min(32, maxiter - it);
    for (int q = 0; q < chunk; ++q) {
      const int iter = ++it;
      // H side (nmf_mu.c:174-191): numerh = W^T A, wtw = W^T W, hden = wtw H, H rule
      hipLaunchKernelGGL(k_gen_prod, grid((long)k * n), dim3(GB), 0, g.st, k, n, m, dW, 1L, (long)m, dA, 1L, (long)m, numh,
                         1L, (long)k);
      hipLaunchKernelGGL(k_gen_prod, grid((long)k * k), dim3(GB), 0, g.st, k, k, m, dW, 1L, (long)m, dW, 1L, (long)m, wtw,
                         1L, (long)k);
      hipLaunchKernelGGL(k_gen_prod, grid((long)k * n), dim3(GB), 0, g.st, k, n, k, wtw, (long)k, 1L, dH, 1L, (long)k, denh,
                         1L, (long)k);
      hipLaunchKernelGGL(k_gen_rule, grid((long)lh), dim3(GB), 0, g.st, (long)lh, dH, numh, denh, g.state);
      // W side (nmf_mu.c:198-216) with the new h: numerw = A h^T, hht = h h^T, wden = W0 hht, W rule
      hipLaunchKernelGGL(k_gen_prod, grid((long)m * k), dim3(GB), 0, g.st, m, k, n, dA, (long)m, 1L, dH, (long)k, 1L, numw,
                         1L, (long)m);
      hipLaunchKernelGGL(k_gen_prod, grid((long)k * k), dim3(GB), 0, g.st, k, k, n, dH, (long)k, 1L, dH, (long)k, 1L, hht,
                         1L, (long)k);
      hipLaunchKernelGGL(k_gen_prod, grid((long)m * k), dim3(GB), 0, g.st, m, k, k, dW, (long)m, 1L, hht, 1L, (long)k, denw,
                         1L, (long)m);
      hipLaunchKernelGGL(k_gen_rule, grid((long)lw), dim3(GB), 0, g.st, (long)lw, dW, numw, denw, g.state);
      hipLaunchKernelGGL(k_gen_check, dim3(1), dim3(GB), 0, g.st, iter, maxiter, stop_rule, k, n, dH, cls, g.state);
    }
    GCHECK(hipGetLastError());
    GCHECK(hipMemcpyAsync(hstate, g.state, sizeof(int) * 4, hipMemcpyDeviceToHost, g.st));
    GCHECK(hipStreamSynchronize(g.st));
    if (hstate[0]) break;
  }
  GCHECK(hipMemcpyAsync(W, dW, lw * sizeof(double), hipMemcpyDeviceToHost, g.st));
  GCHECK(hipMemcpyAsync(H, dH, lh * sizeof(double), hipMemcpyDeviceToHost, g.st));
  GCHECK(hipMemcpyAsync(hstate, g.state, sizeof(int) * 4, hipMemcpyDeviceToHost, g.st));
  GCHECK(hipStreamSynchronize(g.st));
  if (iters) *iters = maxiter == 0 ? 0 : hstate[1];
  if (early) *early = hstate[2] == 1;
  return 0;
}
}  // namespace
