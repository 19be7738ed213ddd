// brunet.hip -- batched Brunet KL-divergence MU restarts (C ABI nmfc_brunet_* in include/nmfc.h).
//
// The per-restart algorithm is the BROAD nmfconsensus / GenePattern NMF.div (Brunet et al. 2004),
// which the reference names at test_nmf.r:29 but does not ship (restated in
// oracle/brunet_oracle.c, parity against the reference unpinned):
//   VP = W H;  H <- (H * (W^T (A / VP)) + eps) / colSums(W)          (k_br_hnum + k_br_hupd)
//   VP = W H;  W <- (W * ((A / VP) H^T) + eps) / rowSums(H)          (k_br_wupd)
//   every stopfreq iterations: per-sample argmax class, stop after stopconv unchanged checks.
// Init per restart: set.seed(seed + i); W <- runif(m k); H <- runif(k n) (R's Mersenne-Twister, k_br_init).
//
// The quotient A / VP is restart-specific, so the per-iteration work is 2 m n divides plus 8 m n k
// flop of rank-k products per restart with nothing to share but A: these are VALU kernels (fp64 FMA
// + IEEE divide, the divide dominating for small k), not MFMA GEMMs.  A is shared by streaming one A
// element per lane and applying it to RG restarts at once; the per-restart W row (H-side) or H column
// (W-side) is wave-uniform: it comes through scalar loads into SGPR operands, or for some ranks through
// LDS tiles read back by broadcast (the per-k SL table below), and no cross-lane reductions are needed.
// Layouts (per k batch of B restarts):
//   Arm [m][n_pad] (sample-contiguous rows), Acm [n][m_pad] (gene-contiguous columns)
//   W   [B][m][K]  (gene-major, k contiguous)    H [B][n][K]  (= libnmf column-major k x n)
//   Gp  [chunk][B][K][n_pad]  split-K partials of W^T (A / VP) over fixed gene chunks
// Every sum's order depends only on (m, n, k): fixed gene chunks, fixed tree reductions, never on
// the batch, the group a restart lands in or the GPU count.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "lane_pool.hpp"
#include "nmfc_tuning.hpp"
#include "rmt.hpp"
#include "../../include/nmfc.h"

void nmfc_set_error(const char* msg);

namespace {

constexpr int BT = 256;
constexpr int BR_KMAX = 16;
constexpr double EPS = 2.220446049250313e-16;   // .Machine$double.eps

void br_err(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void br_err(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  nmfc_set_error(buf);
}

#define BCHECK(expr)                                                                       \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) {                                                                \
      br_err("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
      return -1;                                                                           \
    }                                                                                      \
  } while (0)

long rup(long v, long a) { return (v + a - 1) / a * a; }

struct Buf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t need) {
    if (need <= bytes) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    if (need == 0) return 0;
    hipError_t e = hipMalloc(&p, need);
    if (e != hipSuccess) {
      br_err("hipMalloc(%zu) failed: %s", need, hipGetErrorString(e));
      p = nullptr;
      return -1;
    }
    bytes = need;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// Pinned host staging of one lane (the per-check stop-iteration read-back, the live-restart list, the seeds): the
// small per-iteration copies of four lanes never go through HIP's shared pageable staging path.
struct PinBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t need) {
    if (need <= bytes) return 0;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipHostMalloc(&p, need, hipHostMallocDefault);
    if (e != hipSuccess) {
      br_err("hipHostMalloc(%zu) failed: %s", need, hipGetErrorString(e));
      p = nullptr;
      return -1;
    }
    bytes = need;
    return 0;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// q = a / p from a refined reciprocal r of p: q = a r and one residual correction (Markstein's final step), i.e. the
// compiler's IEEE sequence without its operand-scaling steps (div_scale / div_fmas / div_fixup), which only matter
// near the exponent limits, and without its second Newton step.  r comes from v_rcp_f64 (good to 2^-24.4 on gfx950)
// and one Newton step (~2^-48.8), so the corrected quotient's error is ~2^-97 relative before its rounding: the result
// is FAITHFUL, and it matched the correctly rounded a / p on every one of 3.2e9 random probe pairs (tools/quot_probe.hip,
// a, p over 2^-60..2^10) -- but it is not proven correctly rounded: a quotient can sit closer to a rounding midpoint
// (down to ~2^-106) than the remaining error, and random pairs almost never hit those cases, so bit parity with an IEEE
// divide is unpinned for them.  Parity to the IEEE-divide oracle on the tested sweeps: tests/test_gpu_brunet.py.
// NMFC_BRUNET_IEEEDIV (a build of tools/build_variant.sh) is the exact IEEE option.
__device__ __forceinline__ double quot_r(double a, double p, double r) {
#if NMFC_BRUNET_IEEEDIV
  (void)r;
  return a / p;
#else
  const double q = a * r;
  return fma(fma(-p, q, a), r, q);
#endif
}

// Refined reciprocals of N positive values from ONE v_rcp_f64 (Montgomery's batch inversion): prefix products
// c_i = p_0 ... p_i, u = 1 / c_{N-1} by v_rcp_f64 and one Newton step, then r_i = u c_{i-1} and u <- u p_i from the top
// down (N = 1: v_rcp_f64 + one Newton step, the round-5 sequence).  v_rcp_f64 issues at about a third of the fp64 FMA
// rate on gfx950 (6.9 vs 2.1 ns per wave instruction per SIMD, tools/quot_probe.hip rate mode,
// profiles/r06/brunet_rcp/), so a batch of N trades N - 1 of them for 3 (N - 1) multiplies.  Each r_i carries the
// Newton error plus at most 2 N roundings of 2^-53, so the corrected quotient keeps its ~2^-96 error and stays faithful
// (0 differences from IEEE a / p in 3.2e9 batched probe quotients).  The prefix products must stay normal: with A
// finite, non-negative and at most 2^64 (checked by nmfc_brunet_create) and caller factors in [2^-60, 2^60] (checked by
// nmfc_brunet_run), every VP of the KL updates lies in [eps^2 / T, T] for T = sum(A) <= 2^100 -- the H update makes the
// column sums of W H equal those of A (the W update the row sums), and the eps terms floor W and H at eps over the
// row / column sums whose products are bounded by T -- so a batch of at most BR_RCP_MAX = 5
// values spans at most 2^(5 (104 + 100)) = 2^1020.
constexpr int BR_RCP_MAX = 5;
template <int N>
__device__ __forceinline__ void recip_batch(const double* p, double* r) {
  static_assert(N >= 1 && N <= BR_RCP_MAX, "batch of 1 .. BR_RCP_MAX reciprocals");
  double c[N];
  c[0] = p[0];
#pragma unroll
  for (int i = 1; i < N; ++i) c[i] = c[i - 1] * p[i];
  double u = __builtin_amdgcn_rcp(c[N - 1]);
  u = fma(u, fma(-c[N - 1], u, 1.0), u);
#pragma unroll
  for (int i = N - 1; i > 0; --i) {
    r[i] = u * c[i - 1];
    u = u * p[i];
  }
  r[0] = u;
}

// reciprocals of NQ values in consecutive batches of at most B
template <int NQ, int B>
__device__ __forceinline__ void recips(const double* p, double* r) {
  constexpr int N = NQ < B ? NQ : B;
  recip_batch<N>(p, r);
  if constexpr (NQ > N) recips<NQ - N, B>(p + N, r + N);
}

// Per-rank configuration of the two VALU kernels (tables in nmfc_tuning.hpp, per kernel since round 6):
//  SPL  elements per lane: the LDS return path moves 8K bytes per lane for every element-restart's operand row; where
//       that (rather than the VALU work) bounds the kernel, each row serves 2 elements (k = 8, 9; elsewhere the doubled
//       register state costs more occupancy than the traffic saves: profiles/r01f_brunet_spl.txt).
//  RG   restarts per workgroup: each lane keeps SPL * RG * 4K values of state; RG shares every A element loaded over RG
//       restarts.  The best RG is not monotone in k: register-count occupancy steps and grid size (groups = R / RG)
//       move together (profiles/r01g/brunet_rg/, profiles/r06/brunet_sload/).  RG never changes a restart's arithmetic.
//  SL   the wave-uniform operand rows by scalar loads into SGPR operands instead of the double-buffered LDS tiles: no
//       LDS return-path bytes and no barriers, and the rows leave the VGPRs (occupancy up a step for k >= 4); the same
//       arithmetic in the same order, so the same bits.
//  RCP  the RG * SPL quotients of a lane's gene (sample) step take their reciprocals in batches of at most RCP from one
//       v_rcp_f64 each (recip_batch); 1: one v_rcp_f64 per quotient.
constexpr int br_nib(unsigned long long t, int K) { return K < 16 ? (int)((t >> (4 * K)) & 15) : 0; }
constexpr int rgh_of(int K) { return br_nib(NMFC_BR_RGH, K) ? br_nib(NMFC_BR_RGH, K) : 1; }
constexpr int rgw_of(int K) { return br_nib(NMFC_BR_RGW, K) ? br_nib(NMFC_BR_RGW, K) : 1; }
constexpr int splh_of(int K) { return ((NMFC_BR_SPLH >> K) & 1ULL) ? 2 : 1; }
constexpr int splw_of(int K) { return ((NMFC_BR_SPLW >> K) & 1ULL) ? 2 : 1; }
constexpr bool slh_of(int K) { return (NMFC_BR_SLH >> K) & 1ULL; }
constexpr bool slw_of(int K) { return (NMFC_BR_SLW >> K) & 1ULL; }
constexpr int rcp_clamp(int b) { return b < 1 ? 1 : (b > BR_RCP_MAX ? BR_RCP_MAX : b); }
constexpr int rcph_of(int K) { return rcp_clamp(br_nib(NMFC_BR_RCPH, K)); }
constexpr int rcpw_of(int K) { return rcp_clamp(br_nib(NMFC_BR_RCPW, K)); }
// small batches (B <= NMFC_BR_SMALL_B restarts of one k, e.g. one rank's shard of a strong-scaling
// run): fewer restarts per workgroup so the batch still spreads over the CUs
constexpr int rg_small(int rg) {
  return NMFC_BR_RG_SMALL_DIV == 0 ? 1 : (rg / NMFC_BR_RG_SMALL_DIV > 1 ? rg / NMFC_BR_RG_SMALL_DIV : 1);
}

// ------------------------------------------------------------------------------------------------
// Kernels
// ------------------------------------------------------------------------------------------------

// set.seed(seeds[b]); W <- matrix(runif(m*K), m, K); H <- matrix(runif(K*n), K, n)  (one workgroup per
// restart; R's Mersenne-Twister from rmt.hpp).
__global__ __launch_bounds__(BT) void k_br_init(const uint32_t* __restrict__ seeds, int m, int n, int K,
                                                double* __restrict__ W, long wstride, double* __restrict__ H,
                                                long hstride) {
  __shared__ uint32_t mt[624];
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) rmt::seed_table(mt, seeds[b]);
  __syncthreads();
  const long nw = (long)m * K, total = nw + (long)K * n;
  double* Wb = W + (long)b * wstride;
  double* Hb = H + (long)b * hstride;
  for (long base = 0; base < total; base += 624) {
    rmt::regenerate<BT>(mt);
    for (int t = tid; t < 624; t += BT) {
      const long d = base + t;
      if (d >= total) break;
      const double u = rmt::unif(mt[t]);
      if (d < nw)
        Wb[(d % m) * K + d / m] = u;
      else
        Hb[d - nw] = u;
    }
    __syncthreads();
  }
}

// Tile of the wave-uniform operand (W rows of the H side, H columns of the W side) for the RG
// restarts of a workgroup: TL consecutive gene (sample) rows of K doubles per restart, contiguous in
// HBM, fetched with coalesced vector loads one tile ahead into registers and stored into the other
// half of a double-buffered LDS array; the inner loop reads it back with broadcast LDS reads.
constexpr int TL = NMFC_BR_TL;
// inner-loop unroll per k and kernel (tools/brunet_kbench.py on the C5 shape; unroll 2 where the unrolled live ranges
// push the register count past an occupancy step).  Round 6, re-measured with the per-kernel SL / RG / SPL tables
// against 1 / 2 / 4 / 8 for every k (profiles/r06/brunet_sload/n_*): H side 2 at k = 4 (-5 %), 4 at k = 6 (-8 %), 8 at
// k = 10 (-6.5 %); W side 4 at k = 4 (-4 %), 2 at k = 6; the rest as round 5 (profiles/r05/brunet/kbench_unroll_rg.txt).
constexpr int br_unroll_h(int K) {   // NMFC_BR_UNROLL != 0: one unroll for every k and kernel (experiment builds)
  return NMFC_BR_UNROLL != 0 ? NMFC_BR_UNROLL
                             : K == 10 ? 8 : (K == 4 || K == 5 || K == 7 || K == 8) ? 2 : 4;
}
constexpr int br_unroll_w(int K) {
  return NMFC_BR_UNROLL != 0 ? NMFC_BR_UNROLL : (K == 5 || K == 6 || K == 7 || K == 8 || K == 10) ? 2 : 4;
}

template <int K, int RG>
struct OperandTiles {
  static constexpr int TW = RG * TL * K;              // doubles per tile (all restarts)
  static constexpr int PER = (TW + BT - 1) / BT;      // per thread
  double pre[PER];
  // rows [t0, t0 + TL) of X[slot_r][row][c] (row stride K), rows >= rows_end read as 0
  __device__ __forceinline__ void fetch(const double* __restrict__ X, long stride, const int* sl, int t0,
                                        int rows_end) {
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int idx = threadIdx.x + e * BT;
      double v = 0.0;
      if (idx < TW) {
        const int r = idx / (TL * K), rem = idx - r * (TL * K);
        if (rem < (rows_end - t0) * K) v = X[(long)sl[r] * stride + (long)t0 * K + rem];
      }
      pre[e] = v;
    }
  }
  __device__ __forceinline__ void store(double* lds) {
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int idx = threadIdx.x + e * BT;
      if (idx < TW) lds[idx] = pre[e];
    }
  }
};

// H side, split over fixed gene chunks: Gp[chunk][b][c][j] = sum_{i in chunk} W[b][i][c] * A[i][j] / VP[i][j],
// VP[i][j] = sum_c W[b][i][c] H[b][j][c].  Lane = SPL samples j (H columns and accumulators in
// registers); W rows through the double-buffered LDS tiles.  A broadcast ds_read_b128 still moves
// 1 KiB per wave through the LDS return path, so for larger k each W row read serves SPL = 2 samples.
template <int K, int RG, int SPL, bool SL>
__global__ __launch_bounds__(BT) void k_br_hnum(const double* __restrict__ Arm, long n_pad, int m, int n, int gc,
                                                const int* __restrict__ act, int nact, const double* __restrict__ W,
                                                long wstride, const double* __restrict__ H, long hstride,
                                                double* __restrict__ Gp, long gp_cs) {
  using OT = OperandTiles<K, RG>;
  __shared__ double wl[2][OT::TW];
  __shared__ int sl[RG];
  int jj[SPL], jl[SPL];
#pragma unroll
  for (int s = 0; s < SPL; ++s) {
    jj[s] = blockIdx.x * (BT * SPL) + s * BT + threadIdx.x;
    jl[s] = jj[s] < n ? jj[s] : n - 1;
  }
  const int chunk = blockIdx.y;
  const int g0 = blockIdx.z * RG;
  const int nlive = min(RG, nact - g0);
  const int i0 = chunk * gc, i1 = min(m, i0 + gc);
  if (threadIdx.x < RG) sl[threadIdx.x] = act[min(g0 + (int)threadIdx.x, nact - 1)];
  __syncthreads();
  long wro[RG];   // SL: each restart's W row base, wave-uniform
#pragma unroll
  for (int r = 0; r < RG; ++r) wro[r] = (long)__builtin_amdgcn_readfirstlane(sl[r]) * wstride;
  double h[SPL][RG][K], g[SPL][RG][K];
#pragma unroll
  for (int s = 0; s < SPL; ++s)
#pragma unroll
    for (int r = 0; r < RG; ++r)
#pragma unroll
      for (int c = 0; c < K; ++c) {
        h[s][r][c] = H[(long)sl[r] * hstride + (long)jl[s] * K + c];
        g[s][r][c] = 0.0;
      }
  OT ot;
  if constexpr (!SL) {
    ot.fetch(W, wstride, sl, i0, i1);
    ot.store(wl[0]);
    __syncthreads();
  }
  int buf = 0;
  for (int t0 = i0; t0 < i1; t0 += TL, buf ^= 1) {
    const bool more = !SL && t0 + TL < i1;
    if (more) ot.fetch(W, wstride, sl, t0 + TL, i1);
    const double* ap = Arm + (long)t0 * n_pad;
    const double* wt = wl[buf];
    const double* wg = W + (long)t0 * K;
    // one gene: every quotient's VP first, their reciprocals in batches of rcph_of(K) (recips), then the accumulations
    // (each accumulator still adds its genes in gene order).  Slots past the live restarts repeat the last live one
    // (computed, never stored): no branches here
    auto gene = [&](int ii) {
      constexpr int NQ = RG * SPL;
      double a[SPL], w[RG][K], p[NQ], rr[NQ];
#pragma unroll
      for (int s = 0; s < SPL; ++s) a[s] = ap[(long)ii * n_pad + jl[s]];
#pragma unroll
      for (int r = 0; r < RG; ++r) {
        const double* wr = SL ? wg + wro[r] + ii * K : wt + r * (TL * K) + ii * K;
#pragma unroll
        for (int c = 0; c < K; ++c) w[r][c] = wr[c];
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
          double v = 0.0;
#pragma unroll
          for (int c = 0; c < K; ++c) v = fma(w[r][c], h[s][r][c], v);
          p[r * SPL + s] = v;
        }
      }
      recips<NQ, rcph_of(K)>(p, rr);
#pragma unroll
      for (int r = 0; r < RG; ++r)
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
          const double q = quot_r(a[s], p[r * SPL + s], rr[r * SPL + s]);
#pragma unroll
          for (int c = 0; c < K; ++c) g[s][r][c] = fma(w[r][c], q, g[s][r][c]);
        }
    };
    if (i1 - t0 >= TL) {
#pragma unroll br_unroll_h(K)
      for (int ii = 0; ii < TL; ++ii) gene(ii);
    } else {
      for (int ii = 0; ii < i1 - t0; ++ii) gene(ii);
    }
    if constexpr (!SL) {
      if (more) ot.store(wl[buf ^ 1]);
      __syncthreads();
    }
  }
#pragma unroll
  for (int s = 0; s < SPL; ++s)
    if (jj[s] < n) {
#pragma unroll
      for (int r = 0; r < RG; ++r)
        if (r < nlive) {
#pragma unroll
          for (int c = 0; c < K; ++c) Gp[(long)chunk * gp_cs + ((long)sl[r] * K + c) * n_pad + jj[s]] = g[s][r][c];
        }
    }
}

// The workgroup sum of v[c] in the fixed tree order red[t] += red[t + s], s = BT/2, ..., 1: the strides of 64 and
// more through LDS, the last six inside wave 0 by lane shuffles (lane t adds lane t + s's value of the previous
// step, exactly the LDS tree's operands), so 3 barriers instead of 9 and the same bits.
template <int K>
__device__ __forceinline__ void tree_sum(double (*red)[BT], double* v) {
  static_assert(BT == 256, "tree_sum: two LDS steps then one wave");
  const int tid = threadIdx.x;
#pragma unroll
  for (int c = 0; c < K; ++c) red[c][tid] = v[c];
  __syncthreads();
  if (tid < 128) {
#pragma unroll
    for (int c = 0; c < K; ++c) red[c][tid] += red[c][tid + 128];
  }
  __syncthreads();
  if (tid < 64) {
#pragma unroll
    for (int c = 0; c < K; ++c) {
      double x = red[c][tid] + red[c][tid + 64];
#pragma unroll
      for (int s = 32; s > 0; s >>= 1) x = x + __shfl_down(x, s);
      if (tid == 0) red[c][0] = x;
    }
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < K; ++c) v[c] = red[c][0];
  __syncthreads();
}

// One workgroup per live restart: colSums(W) (apply(W, 2, sum)), sum of the chunk partials,
// H <- (H * G + eps) / colSums(W), rowSums(new H) for the W side, and on check iterations the
// membership test (order(H[,j], decreasing = TRUE)[1] vs the previous check).
template <int K>
__global__ __launch_bounds__(BT) void k_br_hupd(int t, int check, int stopconv, int nchunks, int m, int n, long n_pad,
                                                const int* __restrict__ act, const double* __restrict__ W, long wstride,
                                                double* __restrict__ H, long hstride, const double* __restrict__ Gp,
                                                long gp_cs, double* __restrict__ RS, int* __restrict__ memb,
                                                int* __restrict__ nochange, int* __restrict__ stop_iter) {
  __shared__ double red[K][BT];
  const int b = act[blockIdx.x], tid = threadIdx.x;
  double cs[K];
#pragma unroll
  for (int c = 0; c < K; ++c) cs[c] = 0.0;
  const double* Wb = W + (long)b * wstride;
  // this thread's rows i = tid, tid + BT, ... in order, U rows' loads issued ahead of their adds
  constexpr int U = K <= 8 ? 4 : 2;
  int i = tid;
  for (; i + (U - 1) * BT < m; i += U * BT) {
    double v[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < K; ++c) v[u][c] = Wb[(long)(i + u * BT) * K + c];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < K; ++c) cs[c] += v[u][c];
  }
  for (; i < m; i += BT) {
#pragma unroll
    for (int c = 0; c < K; ++c) cs[c] += Wb[(long)i * K + c];
  }
  tree_sum<K>(red, cs);
  double rs[K];
#pragma unroll
  for (int c = 0; c < K; ++c) rs[c] = 0.0;
  int changed = 0;
  double* Hb = H + (long)b * hstride;
  for (int j = tid; j < n; j += BT) {
    double hv[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
      const double* gp = Gp + ((long)b * K + c) * n_pad + j;
      double g = 0.0;   // the chunk partials in chunk order, eight chunks' loads in flight
      for (int ch0 = 0; ch0 < nchunks; ch0 += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ch0 + u < nchunks ? gp[(long)(ch0 + u) * gp_cs] : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (ch0 + u < nchunks) g += v[u];
      }
      hv[c] = __dadd_rn(__dmul_rn(Hb[(long)j * K + c], g), EPS) / cs[c];
      Hb[(long)j * K + c] = hv[c];
      rs[c] += hv[c];
    }
    if (check) {
      int best = 0;
#pragma unroll
      for (int c = 1; c < K; ++c)
        if (hv[c] > hv[best]) best = c;
      const int mm = best + 1;
      if (mm != memb[(long)b * n + j]) changed = 1;
      memb[(long)b * n + j] = mm;
    }
  }
  tree_sum<K>(red, rs);
  if (tid == 0) {
#pragma unroll
    for (int c = 0; c < K; ++c) RS[(long)b * K + c] = rs[c];
  }
  if (check) {
    const int any = __syncthreads_or(changed);
    if (tid == 0) {
      const int nc = any ? 0 : nochange[b] + 1;
      nochange[b] = nc;
      if (nc == stopconv) stop_iter[b] = t;
    }
  }
}

// W side: lane = SPL genes i over every sample j: F[i][c] = sum_j A[i][j] / VP[i][j] * H[j][c] with the
// new H (LDS tiles of TL samples) and the old W rows in registers; W <- (W * F + eps) / rowSums(H).
template <int K, int RG, int SPL, bool SL>
__global__ __launch_bounds__(BT) void k_br_wupd(const double* __restrict__ Acm, long m_pad, int m, int n,
                                                const int* __restrict__ act, int nact, double* __restrict__ W,
                                                long wstride, const double* __restrict__ H, long hstride,
                                                const double* __restrict__ RS) {
  using OT = OperandTiles<K, RG>;
  __shared__ double hl[2][OT::TW];
  __shared__ int sl[RG];
  int ig[SPL], il[SPL];
#pragma unroll
  for (int s = 0; s < SPL; ++s) {
    ig[s] = blockIdx.x * (BT * SPL) + s * BT + threadIdx.x;
    il[s] = ig[s] < m ? ig[s] : m - 1;
  }
  const int g0 = blockIdx.y * RG;
  const int nlive = min(RG, nact - g0);
  if (threadIdx.x < RG) sl[threadIdx.x] = act[min(g0 + (int)threadIdx.x, nact - 1)];
  __syncthreads();
  long hro[RG];   // SL: each restart's H row base, wave-uniform
#pragma unroll
  for (int r = 0; r < RG; ++r) hro[r] = (long)__builtin_amdgcn_readfirstlane(sl[r]) * hstride;
  double w[SPL][RG][K], f[SPL][RG][K];
#pragma unroll
  for (int s = 0; s < SPL; ++s)
#pragma unroll
    for (int r = 0; r < RG; ++r)
#pragma unroll
      for (int c = 0; c < K; ++c) {
        w[s][r][c] = W[(long)sl[r] * wstride + (long)il[s] * K + c];
        f[s][r][c] = 0.0;
      }
  OT ot;
  if constexpr (!SL) {
    ot.fetch(H, hstride, sl, 0, n);
    ot.store(hl[0]);
    __syncthreads();
  }
  int buf = 0;
  for (int s0 = 0; s0 < n; s0 += TL, buf ^= 1) {
    const bool more = !SL && s0 + TL < n;
    if (more) ot.fetch(H, hstride, sl, s0 + TL, n);
    const double* ap = Acm + (long)s0 * m_pad;
    const double* ht = hl[buf];
    const double* hg = H + (long)s0 * K;
    // one sample, as the H side's gene(): VPs, batched reciprocals, accumulations
    auto sample = [&](int jj) {
      constexpr int NQ = RG * SPL;
      double a[SPL], hh[RG][K], p[NQ], rr[NQ];
#pragma unroll
      for (int s = 0; s < SPL; ++s) a[s] = ap[(long)jj * m_pad + il[s]];
#pragma unroll
      for (int r = 0; r < RG; ++r) {
        const double* hj = SL ? hg + hro[r] + jj * K : ht + r * (TL * K) + jj * K;
#pragma unroll
        for (int c = 0; c < K; ++c) hh[r][c] = hj[c];
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
          double v = 0.0;
#pragma unroll
          for (int c = 0; c < K; ++c) v = fma(w[s][r][c], hh[r][c], v);
          p[r * SPL + s] = v;
        }
      }
      recips<NQ, rcpw_of(K)>(p, rr);
#pragma unroll
      for (int r = 0; r < RG; ++r)
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
          const double q = quot_r(a[s], p[r * SPL + s], rr[r * SPL + s]);
#pragma unroll
          for (int c = 0; c < K; ++c) f[s][r][c] = fma(q, hh[r][c], f[s][r][c]);
        }
    };
    if (n - s0 >= TL) {
#pragma unroll br_unroll_w(K)
      for (int jj = 0; jj < TL; ++jj) sample(jj);
    } else {
      for (int jj = 0; jj < n - s0; ++jj) sample(jj);
    }
    if constexpr (!SL) {
      if (more) ot.store(hl[buf ^ 1]);
      __syncthreads();
    }
  }
#pragma unroll
  for (int s = 0; s < SPL; ++s)
    if (ig[s] < m) {
#pragma unroll
      for (int r = 0; r < RG; ++r)
        if (r < nlive) {
#pragma unroll
          for (int c = 0; c < K; ++c)
            W[(long)sl[r] * wstride + (long)ig[s] * K + c] =
                __dadd_rn(__dmul_rn(w[s][r][c], f[s][r][c]), EPS) / RS[(long)sl[r] * K + c];
        }
    }
}

// labels[b][j] = order(H[,j], decreasing = TRUE)[1] (first row of the column maximum, 1-based)
__global__ __launch_bounds__(BT) void k_br_labels(const double* __restrict__ H, long hstride, int K, int n,
                                                  int32_t* __restrict__ labels) {
  const int b = blockIdx.y, j = blockIdx.x * BT + threadIdx.x;
  if (j >= n) return;
  const double* h = H + (long)b * hstride + (long)j * K;
  int best = 0;
  for (int c = 1; c < K; ++c)
    if (h[c] > h[best]) best = c;
  labels[(long)b * n + j] = best + 1;
}

// connect.matrix[i][j] = sum_b [labels_b(i) == labels_b(j)]   (exact integers)
__global__ __launch_bounds__(BT) void k_br_counts(const int32_t* __restrict__ labels, int B, int n,
                                                  int32_t* __restrict__ counts) {
  const int i = blockIdx.x * 16 + (threadIdx.x & 15);
  const int j = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (i >= n || j >= n) return;
  int32_t cnt = 0;
  for (int b = 0; b < B; ++b) cnt += labels[(long)b * n + i] == labels[(long)b * n + j];
  counts[(long)j * n + i] = cnt;
}

__global__ void k_br_divide(const int32_t* __restrict__ counts, double denom, long len, double* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < len) out[i] = (double)counts[i] / denom;
}

// ... and the domain check of recip_batch: *bad = 1 (a plain store; every writer stores the same value) when an entry
// is not a finite number in [0, 2^64]
__global__ void k_br_layout(const double* __restrict__ A, int m, int n, long m_pad, long n_pad,
                            double* __restrict__ Acm, double* __restrict__ Arm, int* __restrict__ bad) {
  const int i = blockIdx.x * BT + threadIdx.x, j = blockIdx.y;
  if (i >= m) return;
  const double v = A[(long)j * m + i];
  Acm[(long)j * m_pad + i] = v;
  Arm[(long)i * n_pad + j] = v;
  if (!(v >= 0.0 && v <= 0x1p64)) *bad = 1;   // NaN fails both tests
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// Host side.  Each k is one batch of B restarts run by a "lane" (own HIP stream and buffers); up to
// BR_LANES lanes run concurrently from a small host thread pool, largest k first, so that the small
// grids of a batch's last stragglers overlap with the other ranks' batches instead of idling the chip.
// ------------------------------------------------------------------------------------------------
namespace {

constexpr int BR_LANES = 4;   // = the HW queues HIP gives a process by default (GPU_MAX_HW_QUEUES)
enum { BK_HNUM = 0, BK_HUPD = 1, BK_WUPD = 2 };

struct BrLane {
  hipStream_t st = nullptr;
  Buf W, H, Gp, RS, memb, nochange, stop_iter, act, seeds, labels;
  PinBuf h_si, h_act, h_seeds;   // pinned host mirrors of stop_iter, act, seeds
  bool timing = false;
  struct Pending {
    int kid;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> pool;
  double kms[3] = {0, 0, 0};
  long long kcount[3] = {0, 0, 0};
  double kfl_sum[3] = {0, 0, 0};
  void release() {
    Buf* bufs[] = {&W, &H, &Gp, &RS, &memb, &nochange, &stop_iter, &act, &seeds, &labels};
    for (Buf* b : bufs) b->release();
    h_si.release();
    h_act.release();
    h_seeds.release();
    for (auto v : pool) (void)hipEventDestroy(v);
    pool.clear();
    if (st) (void)hipStreamDestroy(st);
    st = nullptr;
  }
};

hipEvent_t br_event(BrLane* L) {
  if (!L->pool.empty()) {
    hipEvent_t v = L->pool.back();
    L->pool.pop_back();
    return v;
  }
  hipEvent_t v = nullptr;
  if (hipEventCreate(&v) != hipSuccess) return nullptr;
  return v;
}

void br_drain(BrLane* L) {
  for (auto& p : L->pending) {
    float ms = 0.f;
    if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) L->kms[p.kid] += ms;
    L->pool.push_back(p.a);
    L->pool.push_back(p.b);
  }
  L->pending.clear();
}

struct BTimed {
  BrLane* L;
  int kid;
  hipEvent_t a = nullptr;
  BTimed(BrLane* L_, int kid_, double flops) : L(L_), kid(kid_) {
    L->kcount[kid] += 1;
    L->kfl_sum[kid] += flops;
    if (L->timing && (a = br_event(L))) (void)hipEventRecord(a, L->st);
  }
  ~BTimed() {
    if (L->timing && a) {
      hipEvent_t b = br_event(L);
      if (b) {
        (void)hipEventRecord(b, L->st);
        L->pending.push_back({kid, a, b});
      }
    }
  }
};

}  // namespace

struct nmfc_brunet {
  int dev = 0;
  hipStream_t st = nullptr;
  int m = 0, n = 0;
  long m_pad = 0, n_pad = 0;
  int gc = 0, nchunks = 0;
  int nlanes = BR_LANES;
  Buf Acm, Arm, counts_tmp, cons_tmp;
  BrLane lanes[BR_LANES];
  bool timing = false;
  double kms[3] = {0, 0, 0};
  long long kcount[3] = {0, 0, 0};
  double kfl_sum[3] = {0, 0, 0};
};

namespace {

// one k: B restarts (slots 0..B-1) already initialised in L->W / L->H; iterates to the stop rule.
template <int K, int RGH = rgh_of(K), int RGW = rgw_of(K)>
int br_iterate(const nmfc_brunet* e, BrLane* L, int B, const nmfc_brunet_opts& o, std::vector<int>& iters,
               std::vector<int>& stopped) {
  constexpr int SPLH = splh_of(K), SPLW = splw_of(K);
  const int m = e->m, n = e->n;
  hipStream_t st = L->st;
  const long wstride = (long)m * K, hstride = (long)n * K;
  const long gp_cs = (long)B * K * e->n_pad;
  int* act = L->h_act.as<int>();   // pinned (br_run_k sized them): host list of live restart slots
  int* si = L->h_si.as<int>();     // pinned read-back of stop_iter
  for (int b = 0; b < B; ++b) act[b] = b, si[b] = 0;
  int nact = B;
  BCHECK(hipMemcpyAsync(L->act.p, act, sizeof(int) * B, hipMemcpyHostToDevice, st));
  BCHECK(hipMemsetAsync(L->memb.p, 0, sizeof(int) * (size_t)B * n, st));   // old.membership starts at 0
  BCHECK(hipMemsetAsync(L->nochange.p, 0, sizeof(int) * B, st));
  BCHECK(hipMemsetAsync(L->stop_iter.p, 0, sizeof(int) * B, st));
  const double fl = 4.0 * m * n * K;   // algorithmic flop per restart and kernel: VP (2mnk) + product (2mnk)
  for (int t = 1; t <= o.maxiter && nact > 0; ++t) {
    const int check = (t % o.stopfreq) == 0;
    const int groups_h = (nact + RGH - 1) / RGH, groups_w = (nact + RGW - 1) / RGW;
    {
      BTimed tl(L, BK_HNUM, fl * nact);
      hipLaunchKernelGGL((k_br_hnum<K, RGH, SPLH, slh_of(K)>), dim3((n + BT * SPLH - 1) / (BT * SPLH), e->nchunks, groups_h),
                         dim3(BT), 0, st,
                         e->Arm.as<double>(), e->n_pad, m, n, e->gc, L->act.as<int>(), nact, L->W.as<double>(), wstride,
                         L->H.as<double>(), hstride, L->Gp.as<double>(), gp_cs);
    }
    {
      BTimed tl(L, BK_HUPD, 0.0);
      hipLaunchKernelGGL((k_br_hupd<K>), dim3(nact), dim3(BT), 0, st, t, check, o.stopconv, e->nchunks, m, n, e->n_pad,
                         L->act.as<int>(), L->W.as<double>(), wstride, L->H.as<double>(), hstride, L->Gp.as<double>(),
                         gp_cs, L->RS.as<double>(), L->memb.as<int>(), L->nochange.as<int>(), L->stop_iter.as<int>());
    }
    {
      BTimed tl(L, BK_WUPD, fl * nact);
      hipLaunchKernelGGL((k_br_wupd<K, RGW, SPLW, slw_of(K)>), dim3((m + BT * SPLW - 1) / (BT * SPLW), groups_w), dim3(BT), 0, st,
                         e->Acm.as<double>(),
                         e->m_pad, m, n, L->act.as<int>(), nact, L->W.as<double>(), wstride, L->H.as<double>(), hstride,
                         L->RS.as<double>());
    }
    BCHECK(hipGetLastError());
    if (check) {
      // stops happen only on check iterations, after that iteration's W update (NMF.div breaks at the
      // end of the iteration): drop stopped restarts from the launch list
      BCHECK(hipMemcpyAsync(si, L->stop_iter.p, sizeof(int) * B, hipMemcpyDeviceToHost, st));
      BCHECK(hipStreamSynchronize(st));
      if (L->timing) br_drain(L);
      int q = 0;
      for (int x = 0; x < nact; ++x)
        if (si[act[x]] == 0) act[q++] = act[x];
      if (q != nact) {
        nact = q;
        if (nact > 0) BCHECK(hipMemcpyAsync(L->act.p, act, sizeof(int) * nact, hipMemcpyHostToDevice, st));
        BCHECK(hipStreamSynchronize(st));
      }
    }
  }
  BCHECK(hipMemcpyAsync(si, L->stop_iter.p, sizeof(int) * B, hipMemcpyDeviceToHost, st));
  BCHECK(hipStreamSynchronize(st));
  if (L->timing) br_drain(L);
  iters.resize(B);
  stopped.resize(B);
  for (int b = 0; b < B; ++b) {
    iters[b] = si[b] ? si[b] : o.maxiter;   // NMF.div returns t: the break iteration, else maxniter
    stopped[b] = si[b] != 0;
  }
  return 0;
}

int br_dispatch(const nmfc_brunet* e, BrLane* L, int K, int B, const nmfc_brunet_opts& o, std::vector<int>& iters,
                std::vector<int>& stopped) {
  switch (K) {
#define BR_CASE(KK) \
  case KK:          \
    return B <= NMFC_BR_SMALL_B ? br_iterate<KK, rg_small(rgh_of(KK)), rg_small(rgw_of(KK))>(e, L, B, o, iters, stopped) \
                                : br_iterate<KK>(e, L, B, o, iters, stopped);
    BR_CASE(2) BR_CASE(3) BR_CASE(4) BR_CASE(5) BR_CASE(6) BR_CASE(7) BR_CASE(8) BR_CASE(9) BR_CASE(10) BR_CASE(11)
    BR_CASE(12) BR_CASE(13) BR_CASE(14) BR_CASE(15) BR_CASE(16)
#undef BR_CASE
    default:
      br_err("nmfc_brunet_run: k=%d unsupported", K);
      return -1;
  }
}

// Everything for one k on one lane: init, iterations, labels, counts slice, host outputs.
struct KJob {
  int ki, K;
  long woff, hoff;   // offsets of this k's jobs in the W / H outputs
};

int br_run_k(nmfc_brunet* e, BrLane* L, const KJob& kj, int B, int R, const nmfc_brunet_opts& o, const double* W_init,
             const double* H_init, int32_t* dcounts, nmfc_result* out, long long* tot_iters, int* max_it) {
  const int m = e->m, n = e->n, K = kj.K, ki = kj.ki;
  BCHECK(hipSetDevice(e->dev));
  if (!L->st) BCHECK(hipStreamCreateWithFlags(&L->st, hipStreamNonBlocking));
  hipStream_t st = L->st;
  if (L->W.ensure(sizeof(double) * (size_t)B * m * K) || L->H.ensure(sizeof(double) * (size_t)B * n * K) ||
      L->Gp.ensure(sizeof(double) * (size_t)e->nchunks * B * K * e->n_pad) ||
      L->RS.ensure(sizeof(double) * (size_t)B * K) || L->memb.ensure(sizeof(int) * (size_t)B * n) ||
      L->nochange.ensure(sizeof(int) * B) || L->stop_iter.ensure(sizeof(int) * B) || L->act.ensure(sizeof(int) * B) ||
      L->seeds.ensure(sizeof(uint32_t) * B) || L->labels.ensure(sizeof(int32_t) * (size_t)B * n) ||
      L->h_si.ensure(sizeof(int) * B) || L->h_act.ensure(sizeof(int) * B) || L->h_seeds.ensure(sizeof(uint32_t) * B))
    return -1;
  const long wstride = (long)m * K, hstride = (long)n * K;
  std::vector<double> hw, hh;
  uint32_t* seeds = L->h_seeds.as<uint32_t>();
  const int rb = std::max(0, o.restart_begin);
  for (int b = 0; b < B; ++b) seeds[b] = o.seed + (uint32_t)(rb + b + 1);   // set.seed(rseed + i), i 1-based
  BCHECK(hipMemcpyAsync(L->seeds.p, seeds, sizeof(uint32_t) * B, hipMemcpyHostToDevice, st));
  if (W_init && H_init) {
    // caller factors for this k's B jobs: W_b m x K column-major, H_b K x n column-major; positive and within
    // [2^-60, 2^60] (the batched reciprocals' domain, recip_batch)
    const size_t nwk = (size_t)B * m * K, nhk = (size_t)B * n * K;
    for (size_t x = 0; x < nwk + nhk; ++x) {
      const double v = x < nwk ? W_init[kj.woff + x] : H_init[kj.hoff + (x - nwk)];
      if (!(v >= 0x1p-60 && v <= 0x1p60)) {
        br_err("nmfc_brunet_run: caller factors must lie in [2^-60, 2^60] (k=%d: %g)", K, v);
        return -1;
      }
    }
    hw.assign((size_t)B * m * K, 0.0);
    for (int b = 0; b < B; ++b)
      for (int c = 0; c < K; ++c)
        for (int i = 0; i < m; ++i)
          hw[(size_t)b * wstride + (size_t)i * K + c] = W_init[kj.woff + (long)b * wstride + (long)c * m + i];
    BCHECK(hipMemcpyAsync(L->W.p, hw.data(), sizeof(double) * hw.size(), hipMemcpyHostToDevice, st));
    BCHECK(hipMemcpyAsync(L->H.p, H_init + kj.hoff, sizeof(double) * (size_t)B * hstride, hipMemcpyHostToDevice, st));
  } else {
    hipLaunchKernelGGL(k_br_init, dim3(B), dim3(BT), 0, st, L->seeds.as<uint32_t>(), m, n, K, L->W.as<double>(), wstride,
                       L->H.as<double>(), hstride);
    BCHECK(hipGetLastError());
  }
  BCHECK(hipStreamSynchronize(st));   // seeds / hw host buffers
  std::vector<int> iters, stopped;
  if (br_dispatch(e, L, K, B, o, iters, stopped)) return -1;
  hipLaunchKernelGGL(k_br_labels, dim3((n + BT - 1) / BT, B), dim3(BT), 0, st, L->H.as<double>(), hstride, K, n,
                     L->labels.as<int32_t>());
  BCHECK(hipGetLastError());
  if (dcounts) {
    hipLaunchKernelGGL(k_br_counts, dim3((n + 15) / 16, (n + 15) / 16), dim3(BT), 0, st, L->labels.as<int32_t>(), B, n,
                       dcounts + (size_t)n * n * ki);
    BCHECK(hipGetLastError());
  }
  if (out && out->labels)
    BCHECK(hipMemcpyAsync(out->labels + (size_t)ki * B * n, L->labels.p, sizeof(int32_t) * (size_t)B * n,
                          hipMemcpyDeviceToHost, st));
  if (out && (out->W || out->H)) {
    hw.resize((size_t)B * wstride);
    hh.resize((size_t)B * hstride);
    BCHECK(hipMemcpyAsync(hw.data(), L->W.p, sizeof(double) * hw.size(), hipMemcpyDeviceToHost, st));
    BCHECK(hipMemcpyAsync(hh.data(), L->H.p, sizeof(double) * hh.size(), hipMemcpyDeviceToHost, st));
    BCHECK(hipStreamSynchronize(st));
    if (out->W)
      for (int b = 0; b < B; ++b)
        for (int c = 0; c < K; ++c)
          for (int i = 0; i < m; ++i)
            out->W[kj.woff + (long)b * wstride + (long)c * m + i] = hw[(size_t)b * wstride + (size_t)i * K + c];
    if (out->H) memcpy(out->H + kj.hoff, hh.data(), sizeof(double) * hh.size());
  }
  BCHECK(hipStreamSynchronize(st));
  for (int b = 0; b < B; ++b) {
    *tot_iters += iters[b];
    *max_it = std::max(*max_it, iters[b]);
    if (out && out->iters) out->iters[(size_t)ki * B + b] = iters[b];
    if (out && out->stopped_early) out->stopped_early[(size_t)ki * B + b] = stopped[b];
  }
  return 0;
}

}  // namespace

extern "C" {

const char* nmfc_build_tuning_brunet(void) { return NMFC_TUNING_BRUNET; }

void nmfc_brunet_default_opts(nmfc_brunet_opts* o) {
  memset(o, 0, sizeof *o);
  o->maxiter = 2000;        // NMF.div maxniter
  o->stopconv = 40;         // nmfconsensus stopconv
  o->stopfreq = 10;         // nmfconsensus stopfreq
  o->seed = 123456789u;     // nmfconsensus rseed
  o->restart_begin = 0;
  o->restart_end = -1;
  o->verbose = 0;
}

nmfc_brunet* nmfc_brunet_create(int device, const double* A, int m, int n, int a_on_device) {
  if (!A || m <= 0 || n <= 0) {
    br_err("nmfc_brunet_create: bad arguments (A=%p m=%d n=%d)", (const void*)A, m, n);
    return nullptr;
  }
  nmfc_brunet* e = new nmfc_brunet();
  auto fail = [&](const char* what, hipError_t err) -> nmfc_brunet* {
    br_err("nmfc_brunet_create: %s: %s", what, hipGetErrorString(err));
    nmfc_brunet_destroy(e);
    return nullptr;
  };
  hipError_t err;
  if (device >= 0 && (err = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", err);
  if ((err = hipGetDevice(&e->dev)) != hipSuccess) return fail("hipGetDevice", err);
  if ((err = hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking)) != hipSuccess) return fail("hipStreamCreate", err);
  if (const char* s = getenv("NMFC_BRUNET_LANES")) e->nlanes = std::max(1, std::min(BR_LANES, atoi(s)));
  e->m = m;
  e->n = n;
  e->m_pad = rup(m, BT);
  e->n_pad = rup(n, BT);
  // fixed gene chunks (a function of m only): about 16 chunks of whole LDS tiles, at most 2048 genes
  e->gc = (int)std::min<long>(2048, std::max<long>(TL, rup((m + 15) / 16, TL)));
  e->nchunks = (m + e->gc - 1) / e->gc;
  if (e->Acm.ensure(sizeof(double) * e->m_pad * n) || e->Arm.ensure(sizeof(double) * (size_t)m * e->n_pad)) {
    nmfc_brunet_destroy(e);
    return nullptr;
  }
  if ((err = hipMemsetAsync(e->Acm.p, 0, e->Acm.bytes, e->st)) != hipSuccess) return fail("memset", err);
  if ((err = hipMemsetAsync(e->Arm.p, 0, e->Arm.bytes, e->st)) != hipSuccess) return fail("memset", err);
  const double* dA = A;
  Buf tmp;
  if (!a_on_device) {
    if (tmp.ensure(sizeof(double) * (size_t)m * n)) {
      nmfc_brunet_destroy(e);
      return nullptr;
    }
    if ((err = hipMemcpyAsync(tmp.p, A, sizeof(double) * (size_t)m * n, hipMemcpyHostToDevice, e->st)) != hipSuccess)
      return fail("upload A", err);
    dA = tmp.as<double>();
  }
  Buf dbad;
  if (dbad.ensure(sizeof(int))) {
    nmfc_brunet_destroy(e);
    return nullptr;
  }
  if ((err = hipMemsetAsync(dbad.p, 0, sizeof(int), e->st)) != hipSuccess) return fail("memset", err);
  hipLaunchKernelGGL(k_br_layout, dim3((m + BT - 1) / BT, n), dim3(BT), 0, e->st, dA, m, n, e->m_pad, e->n_pad,
                     e->Acm.as<double>(), e->Arm.as<double>(), dbad.as<int>());
  if ((err = hipGetLastError()) != hipSuccess) return fail("k_br_layout", err);
  int bad = 0;
  if ((err = hipMemcpyAsync(&bad, dbad.p, sizeof(int), hipMemcpyDeviceToHost, e->st)) != hipSuccess)
    return fail("read-back", err);
  if ((err = hipStreamSynchronize(e->st)) != hipSuccess) return fail("sync", err);
  tmp.release();
  dbad.release();
  if (bad) {
    // the KL updates need A >= 0; the bound keeps the batched reciprocals' products normal (recip_batch)
    br_err("nmfc_brunet_create: A must hold finite, non-negative entries of at most 2^64");
    nmfc_brunet_destroy(e);
    return nullptr;
  }
  return e;
}

int nmfc_brunet_device(const nmfc_brunet* e) { return e ? e->dev : -1; }

void nmfc_brunet_destroy(nmfc_brunet* e) {
  if (!e) return;
  if (e->st) (void)hipStreamSynchronize(e->st);
  for (BrLane& L : e->lanes) {
    if (L.st) (void)hipStreamSynchronize(L.st);
    br_drain(&L);
    L.release();
  }
  Buf* bufs[] = {&e->Acm, &e->Arm, &e->counts_tmp, &e->cons_tmp};
  for (Buf* b : bufs) b->release();
  if (e->st) (void)hipStreamDestroy(e->st);
  delete e;
}

void nmfc_brunet_set_timing(nmfc_brunet* e, int enable) {
  if (e) e->timing = enable != 0;
}

long long nmfc_brunet_kernel_time(nmfc_brunet* e, int kid, double* ms_out, double* flops_per_launch) {
  if (!e || kid < 0 || kid > 2) return -1;
  if (ms_out) *ms_out = e->kms[kid];
  if (flops_per_launch) *flops_per_launch = e->kcount[kid] ? e->kfl_sum[kid] / e->kcount[kid] : 0.0;
  return e->kcount[kid];
}

int nmfc_brunet_run(nmfc_brunet* e, const int* ks, int nk, int R, const nmfc_brunet_opts* opts_in,
                    const double* W_init, const double* H_init, nmfc_result* out) {
  if (!e || !ks || nk <= 0 || R <= 0) {
    br_err("nmfc_brunet_run: bad arguments");
    return -1;
  }
  nmfc_brunet_opts o;
  if (opts_in)
    o = *opts_in;
  else
    nmfc_brunet_default_opts(&o);
  const int m = e->m, n = e->n;
  if (o.maxiter < 1 || o.stopfreq < 1 || o.stopconv < 1) {
    br_err("nmfc_brunet_run: maxiter, stopfreq and stopconv must be >= 1");
    return -1;
  }
  for (int q = 0; q < nk; ++q)
    if (ks[q] < 2 || ks[q] > BR_KMAX) {
      br_err("nmfc_brunet_run: k=%d unsupported (need 2 <= k <= %d)", ks[q], BR_KMAX);
      return -1;
    }
  const int rb = std::max(0, o.restart_begin);
  const int re = o.restart_end < 0 ? R : std::min(o.restart_end, R);
  if (rb >= re) {
    br_err("nmfc_brunet_run: empty restart range [%d, %d)", rb, re);
    return -1;
  }
  o.restart_begin = rb;
  const int B = re - rb;
  BCHECK(hipSetDevice(e->dev));
  auto t0 = std::chrono::steady_clock::now();
  int32_t* dcounts = nullptr;
  const size_t nn = (size_t)n * n;
  if (out && (out->counts || out->consensus)) {
    if (out->counts && out->counts_on_device) {
      dcounts = out->counts;
    } else {
      if (e->counts_tmp.ensure(sizeof(int32_t) * nn * nk)) return -1;
      dcounts = e->counts_tmp.as<int32_t>();
    }
  }
  // jobs: output offsets in nmfconsensus order; executed largest k first
  std::vector<KJob> jobs(nk);
  long woff = 0, hoff = 0;
  for (int ki = 0; ki < nk; ++ki) {
    jobs[ki] = {ki, ks[ki], woff, hoff};
    woff += (long)B * m * ks[ki];
    hoff += (long)B * n * ks[ki];
  }
  std::vector<KJob> order(jobs);
  std::stable_sort(order.begin(), order.end(), [](const KJob& a, const KJob& b) { return a.K > b.K; });
  const int nl = std::min(o.lanes > 0 ? std::min(o.lanes, BR_LANES) : e->nlanes, nk);
  std::vector<long long> lane_iters(nl, 0);
  std::vector<int> lane_max(nl, 0);
  for (int l = 0; l < nl; ++l) {
    BrLane& L = e->lanes[l];
    L.timing = e->timing;
    for (int q = 0; q < 3; ++q) L.kms[q] = 0, L.kcount[q] = 0, L.kfl_sum[q] = 0;
  }
  // the k batches, largest first, on nl lanes (csrc/lane_pool.hpp; the scheduler alone runs under TSan in the CPU
  // suite): a lane touches only its own BrLane, its lane_iters / lane_max slot and the outputs of its k
  std::string first_err;
  const int rc = nmfc_host::run_lanes(
      nl, nk,
      [&](int l, int idx) {
        return br_run_k(e, &e->lanes[l], order[idx], B, R, o, W_init, H_init, dcounts, out, &lane_iters[l], &lane_max[l]);
      },
      [] { return std::string(nmfc_last_error()); }, &first_err);
  if (rc) {
    nmfc_set_error(first_err.c_str());
    return -1;
  }
  long long tot_iters = 0;
  int max_it = 0;
  for (int q = 0; q < 3; ++q) e->kms[q] = 0, e->kcount[q] = 0, e->kfl_sum[q] = 0;
  for (int l = 0; l < nl; ++l) {
    tot_iters += lane_iters[l];
    max_it = std::max(max_it, lane_max[l]);
    for (int q = 0; q < 3; ++q) {
      e->kms[q] += e->lanes[l].kms[q];
      e->kcount[q] += e->lanes[l].kcount[q];
      e->kfl_sum[q] += e->lanes[l].kfl_sum[q];
    }
  }
  hipStream_t st = e->st;
  if (out && dcounts) {
    if (out->consensus) {
      if (e->cons_tmp.ensure(sizeof(double) * nn * nk)) return -1;
      hipLaunchKernelGGL(k_br_divide, dim3((unsigned)((nn * nk + BT - 1) / BT)), dim3(BT), 0, st, dcounts, (double)R,
                         (long)(nn * nk), e->cons_tmp.as<double>());
      BCHECK(hipGetLastError());
      BCHECK(hipMemcpyAsync(out->consensus, e->cons_tmp.p, sizeof(double) * nn * nk, hipMemcpyDeviceToHost, st));
    }
    if (out->counts && !out->counts_on_device)
      BCHECK(hipMemcpyAsync(out->counts, dcounts, sizeof(int32_t) * nn * nk, hipMemcpyDeviceToHost, st));
  }
  BCHECK(hipStreamSynchronize(st));
  auto t1 = std::chrono::steady_clock::now();
  if (out) {
    out->seconds_total = std::chrono::duration<double>(t1 - t0).count();
    out->seconds_iterate = out->seconds_total;
    out->restart_iterations = tot_iters;
    out->max_iter_run = max_it;
  }
  if (o.verbose)
    fprintf(stderr, "[nmfc brunet] %d restarts x %d k on %d lanes, mean iters %.1f, max %d, %.3f s\n", B, nk, nl,
            (double)tot_iters / ((double)B * nk), max_it, std::chrono::duration<double>(t1 - t0).count());
  return 0;
}

}  // extern "C"
