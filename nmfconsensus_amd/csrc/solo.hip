// solo.hip -- nmf_mu for ONE restart of rank k = 2..4 on a small matrix (m <= 1024 genes, n <= 40 samples: the
// bundled gct and data sets of its size), run by ONE workgroup (8 waves, one CU) through the whole MU loop and
// the stop rule in one launch (nmf_mu.c:174-282).  The team kernel (k_team_mu) spreads such a restart over 16
// CUs and pays three cross-XCD store -> load trips per iteration (~3.7 us of its 6.4 us at k = 2); one CU holds
// the whole problem instead: A (320 KB at 1000 x 40) lives in the register file for the whole launch.
//
// Layout (4x4x4 f64 MFMA, 4 blocks b of 4 x 4 outputs, K = 4; lane 16 K + 4 b + i holds operand X_b[i][K] and
// Y_b[K][i], result lane 16 i + 4 b + j holds D_b[i][j] -- profiles/r03/mfma_f64_4x4x4_probe.txt):
//   lane l of wave w:  K = l >> 4, b = (l >> 2) & 3, j = l & 3;  gene(s) = 128 w + 16 s + 4 b + K, s < 8
//   a_[s][cg] = A[gene(s)][4 cg + j]        (Y operand of G = W^T A: the reduction runs over genes)
//   w_[s]     = W[gene(s)][j]               (X operand of G and of W^T W; j is the factor row a)
// so G needs no data movement, with no padding of k beyond 4 (the 16x16x4 form pads k to 16).  F = A h^T
// reduces over samples instead, which this layout spreads over the 4 lanes j of a quad and the 10 registers
// cg: VALU fma chains over cg, then a quad butterfly (DPP); E = W0 (h h^T) and the W rule likewise per lane.
// h h^T: three 4x4x4 MFMAs per wave over the 48 padded samples plus a 4-block butterfly, redundantly in
// every wave (no barrier).  Per iteration: G / W^T W MFMAs -> LDS partials | barrier | wave and gene-block
// sums in order | barrier | H update | barrier | stop check (wave 0) + h h^T, F, E, W rule (every wave).
// Every reduction order is a function of (m, n, k) only: deterministic.  Stop rules and outputs as
// nmfc_engine_mu1 (REF_COMPAT windows / ARGMAX_STABLE classes, stop iteration and reason).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "../../include/nmfc.h"
#include "nmfc_kernels.hpp"

void nmfc_set_error(const char* msg);

namespace {

using nmfc::mu_rule;

constexpr int SOLO_W = 8;                        // waves (two per SIMD)
constexpr int SOLO_S = 8;                        // 16-gene steps per wave
constexpr int SOLO_MMAX = SOLO_W * SOLO_S * 16;  // 1024 genes
constexpr int SOLO_NMAX = 40;                    // samples (10 column groups of 4 in registers)
constexpr int SOLO_NCOLP = 48;                   // H columns in LDS (h h^T: 3 MFMA steps of 16 samples)

template <int NCG>
struct SoloSmem {
  // wave partials of G (cg < NCG) and W^T W (NCG) in the MFMA D layout, 64 doubles per (wave, cg); the wave
  // stride is padded by 4 doubles so the four waves a summing quad reads fall in different LDS banks
  double Gp[SOLO_W][(NCG + 1) * 64 + 4];
  double Hc[2][SOLO_NCOLP][4];      // H by (sample, row), rows padded to 4: zero past k and n
  double Gs[4][4 * NCG];            // G = W^T A
  double WW[4][4];                  // W^T W
  int stop, reason;
};

// v from the lane given by the quad permutation CTRL (DPP, two 32-bit moves)
// (mov_dpp: no "old" operand to materialise; quad permutations never read outside the quad)
template <int CTRL>
__device__ __forceinline__ double qdpp(double v) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)(u & 0xffffffffLL), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// nmfc::mu_rule without the early return (no divergent branch around the divide): the same operations in the
// same order, so the same bits
__device__ __forceinline__ double mu_rule_nb(double old, double num, double den) {
  const double q = num / (den + nmfc::DIV_BY_ZERO_AVOIDANCE);
  const double t = old * q;
  return (old == 0.0 || num == 0.0 || t < 0.0) ? 0.0 : t;
}
__device__ __forceinline__ double qbcast(double v, int b) {   // lane b of the quad (b a compile-time constant)
  switch (b) {
    case 0: return qdpp<0x00>(v);
    case 1: return qdpp<0x55>(v);
    case 2: return qdpp<0xAA>(v);
    default: return qdpp<0xFF>(v);
  }
}

// SKIP != 0 only in tools/solobench.hip (phase costs): bit 0 no G / W^T W MFMAs, 1 no F / E / W rule, 2 no h h^T,
// 3 no stop check, 4 no partial sums, 6 phase clock stamps of wave 0 into prof[1..7].
// SL: the last SL gene steps of A live in LDS instead of registers (k >= 3 at n = 40: A's registers would spill)
// Operand layout of a launch.  One restart (nmfc_mu_solo): A m x n column-major (a_ld = m), W m x KK (w_ld = m),
// H KK x n column-major (h_sc = KK, h_sa = 1), the stop state in state[0..1].  A batch (nmfc_engine_run, one
// workgroup per restart): A = the engine's column-major Acm (a_ld = m_pad), W/H the stacked [cols][m_pad] /
// [cols][n_pad] buffers at each job's col0 (w_ld = m_pad, h_sc = 1, h_sa = n_pad), the stop state in
// stop_iter / stop_reason[rid].  Only pointers and strides differ: every arithmetic step is the same code.
struct SoloLayout {
  long a_ld, w_ld, h_sc, h_sa;
  const nmfc::SoloJob* jobs;   // nullptr: one restart
  int* stop_iter;
  int* stop_reason;
  int njobs;                   // batched: jobs in `jobs` (the grid may hold fewer workgroups)
};

// JOBS: the batched form's job loop (its registers stay out of the single-restart form, whose gct k = 2 case is at
// the 256-VGPR edge); both forms run the same arithmetic.
template <int NCG, int SL>
using SoloAl = double[SL > 0 ? SL : 1][NCG][64 * SOLO_W];   // A's gene steps SR.. in LDS, lane-contiguous

// The kernel body; its LDS comes from the caller (the kernel's own __shared__ arrays, or the fused batch kernel's
// buffer), its jobs are jx0, jx0 + jstep, ... of lay.jobs (JOBS) or the one restart.
template <int NCG, int KK, int SKIP, int SBO, int SL, bool JOBS, bool ONE = false>
__device__ __forceinline__ void solo_mu_body(const double* __restrict__ A, int m, int n, double* __restrict__ W,
                                             double* __restrict__ H, int maxiter, int stop_rule,
                                             int* __restrict__ state, int kt_arg, long long* __restrict__ prof,
                                             const SoloLayout& lay, SoloSmem<NCG>& sm, SoloAl<NCG, SL>& Al, int jx0,
                                             int jstep) {
  // gene steps per F batch: larger means fewer H reads from LDS but more live registers (A holds most of them)
  constexpr int SB = SBO ? SBO : KK == 2 ? 8 : 4;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, K = l >> 4, bq = (l >> 2) & 3, j = l & 3;
  // KK = 4: H in LDS by sample c with its rows rotated by c (row a at position (a - c) & 3), so lane j (samples
  // c = j mod 4) finds row (j + r) & 3 at position r: the F accumulation is rotated by lane and its quad reduction
  // needs no selects (as k_solo8_mu)
  constexpr bool ROT = KK == 4;
  auto hp = [](int c, int a) -> int { return ROT ? ((a - c) & 3) : a; };
  constexpr int SR = SOLO_S - SL;   // gene steps of A in registers
  double a_[SR > 0 ? SR : 1][NCG], w_[SOLO_S];
  // A[gene(s)][4 cg + j] from registers (s < SR) or LDS; s, cg compile-time after unrolling
  auto av = [&](int s, int cg) -> double { return s < SR ? a_[s < SR ? s : 0][cg] : Al[s < SR ? 0 : s - SR][cg][tid]; };
  // A once per workgroup: a batched workgroup runs its jobs one after another on the same A
#pragma unroll
  for (int s = 0; s < SOLO_S; ++s) {
    const int g = 128 * w + 16 * s + 4 * bq + K;
#pragma unroll
    for (int cg = 0; cg < NCG; ++cg) {
      const int c = 4 * cg + j;
      const double v = (g < m && c < n) ? A[(long)c * lay.a_ld + g] : 0.0;
      if (s < SR)
        a_[s < SR ? s : 0][cg] = v;
      else
        Al[s < SR ? 0 : s - SR][cg][tid] = v;
    }
  }
  // batched: jobs jx0, jx0 + jstep, ... (the grid may be smaller than the job list, so the solo launches leave CUs
  // to the kernels beside them); one restart otherwise
  const int njobs = JOBS ? lay.njobs : 1;
  for (int jx = JOBS ? jx0 : 0; jx < (ONE ? jx0 + 1 : njobs); jx += JOBS ? jstep : 1) {   // ONE: job jx0 only
  double* __restrict__ Wj = W;
  double* __restrict__ Hj = H;
  int kt = kt_arg, rid = -1;
  if constexpr (JOBS) {
    const nmfc::SoloJob jb = lay.jobs[jx];
    Wj = W + (long)jb.col0 * lay.w_ld;
    Hj = H + (long)jb.col0 * lay.h_sa;
    kt = jb.k;
    rid = jb.rid;
  }
#pragma unroll
  for (int s = 0; s < SOLO_S; ++s) {
    const int g = 128 * w + 16 * s + 4 * bq + K;
    w_[s] = (g < m && j < kt) ? Wj[(long)j * lay.w_ld + g] : 0.0;   // rows kt .. KK - 1: zero padding
  }
  __syncthreads();   // the previous job's last reads of sm are done
  for (int x = tid; x < 2 * SOLO_NCOLP * 4; x += 64 * SOLO_W) (&sm.Hc[0][0][0])[x] = 0.0;
  if (tid == 0) {
    sm.stop = 0;
    sm.reason = 0;
  }
  __syncthreads();
  for (int x = tid; x < kt * n; x += 64 * SOLO_W) {
    const int c = x / kt, a = x - c * kt;
    sm.Hc[0][c][hp(c, a)] = Hj[(long)c * lay.h_sc + (long)a * lay.h_sa];
  }
  __syncthreads();
  long long pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pt = 0;
#define SOLO_STAMP(i)                                             \
  if ((SKIP & 64) && tid == 0) {                                  \
    const long long t_ = (long long)__builtin_readcyclecounter(); \
    if ((i) > 0) pacc[(i)] += t_ - pt;                            \
    pt = t_;                                                      \
  }
  int hb = 0;
  int cls = 0, unch = 0;   // wave 0: lane i's class (REF_COMPAT window i, ARGMAX_STABLE sample i), unchanged checks
  for (int iter = 1; maxiter >= 1 && iter <= maxiter + 1; ++iter) {
    SOLO_STAMP(0);
    // ---- this wave's partials of G = W^T A and W^T W (MFMA chains in gene order) ----
    {
      double acc[NCG + 1];
#pragma unroll
      for (int cg = 0; cg <= NCG; ++cg) acc[cg] = 0.0;
#pragma unroll
      for (int s = 0; s < ((SKIP & 1) ? 0 : SOLO_S); ++s) {
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg) acc[cg] = __builtin_amdgcn_mfma_f64_4x4x4f64(w_[s], av(s, cg), acc[cg], 0, 0, 0);
        acc[NCG] = __builtin_amdgcn_mfma_f64_4x4x4f64(w_[s], w_[s], acc[NCG], 0, 0, 0);
      }
#pragma unroll
      for (int cg = 0; cg <= NCG; ++cg) sm.Gp[w][cg * 64 + l] = acc[cg];
    }
    SOLO_STAMP(1);
    __syncthreads();
    SOLO_STAMP(2);
    if (sm.stop) break;   // decided at the previous iteration (its updates are done)
    // ---- sums: G (k x n) and W^T W (k x k), four threads per entry (a quad): lane p sums waves 2p, 2p + 1
    // (gene blocks b in order), then the quad butterfly ((p0 + p1) + (p2 + p3)) ----
    {
      const int p = tid & 3;
      for (int o = tid >> 2; !(SKIP & 16) && o < KK * n + KK * KK; o += 16 * SOLO_W) {   // whole quads (DPP below)
        int a, c, cg, idx;
        if (o < KK * n) {
          a = o / n;
          c = o - a * n;
          cg = c >> 2;
          idx = 16 * a + (c & 3);
        } else {
          a = (o - KK * n) / KK;
          c = (o - KK * n) - a * KK;
          cg = NCG;
          idx = 16 * a + c;
        }
        const double* g0 = &sm.Gp[2 * p][cg * 64 + idx];
        const double* g1 = &sm.Gp[2 * p + 1][cg * 64 + idx];
        double v = ((g0[0] + g0[4]) + g0[8]) + g0[12];
        v = (((v + g1[0]) + g1[4]) + g1[8]) + g1[12];
        v = v + qdpp<0xB1>(v);
        v = v + qdpp<0x4E>(v);
        if (p == 0) {
          if (o < KK * n)
            sm.Gs[a][c] = v;
          else
            sm.WW[a][c] = v;
        }
      }
    }
    SOLO_STAMP(3);
    __syncthreads();
    // ---- H update (nmf_mu.c:178-191): d = (W^T W) H summed over the rows in order ----
    const int nb = hb ^ 1;
    for (int x = tid; x < KK * n; x += 64 * SOLO_W) {
      const int c = x / KK, a = x - c * KK;
      double d = 0.0;
#pragma unroll
      for (int b = 0; b < KK; ++b) d = fma(sm.WW[a][b], sm.Hc[hb][c][hp(c, b)], d);
      sm.Hc[nb][c][hp(c, a)] = mu_rule(sm.Hc[hb][c][hp(c, a)], sm.Gs[a][c], d);
    }
    __syncthreads();
    SOLO_STAMP(4);
    hb = nb;
    // ---- stop rule (nmf_mu.c:253-282), wave 0; read by every wave after the next iteration's first barrier ----
    if (w == 0) {
      const bool check = !(SKIP & 8) && stop_rule != nmfc::STOP_FIXED && iter > 1 && (iter % 2 == 0);
      int reason = 0;
      if (check) {
        bool ch = false;
        if (stop_rule == nmfc::STOP_REF_COMPAT) {
          // window i reads the flat k x n column-major buffer at [i n, i n + k)
          // (kt: the restart's rank; KK = 4 > kt runs it with zero padding rows, which the rule never reads)
          if (l < kt && l < n) {
            int cl = 0;
            double prev = 0.0;
            for (int jj = 0; jj < kt; ++jj) {
              const int f = l * n + jj, c = f / kt, a = f - c * kt;
              const double v = sm.Hc[hb][c][hp(c, a)];
              if (jj > 0 && v > prev) cl = jj;
              prev = v;
            }
            ch = cl != cls;
            cls = cl;
          }
        } else if (stop_rule == nmfc::STOP_ARGMAX_STABLE) {
          if (l < n) {
            int best = 0;
            double bv = sm.Hc[hb][l][hp(l, 0)];
            for (int a = 1; a < kt; ++a) {
              const double v = sm.Hc[hb][l][hp(l, a)];
              if (v > bv) {
                bv = v;
                best = a;
              }
            }
            ch = best != cls;
            cls = best;
          }
        }
        if (__ballot(ch) == 0) {
          if (++unch >= 200) reason = 1;   // nmf_mu.c:269-271
        } else {
          unch = 0;
        }
      }
      if (!reason && iter >= maxiter) reason = 2;
      if (reason && l == 0) {
        sm.stop = iter;
        sm.reason = reason;
      }
    }
    // ---- h h^T (4x4x4 MFMAs over the samples of block b, then the blocks in order), every wave ----
    double hh = 0.0;
#pragma unroll
    for (int t = 0; t < ((SKIP & 4) ? 0 : SOLO_NCOLP / 16); ++t) {
      const double x = sm.Hc[hb][16 * t + 4 * bq + K][ROT ? ((j - K) & 3) : j];   // row j of the sample
      hh = __builtin_amdgcn_mfma_f64_4x4x4f64(x, x, hh, 0, 0, 0);
    }
    // blocks summed by DPP row rotations; only lanes with b = 0 are read below, where the order is
    // (b0 + b1) + (b2 + b3)
    {
      const long long u = __double_as_longlong(hh);
      const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)(u & 0xffffffffLL), 0x124, 0xF, 0xF, true);   // row_ror:4
      const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), 0x124, 0xF, 0xF, true);
      hh += __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
      const long long v = __double_as_longlong(hh);
      const int lo2 = __builtin_amdgcn_mov_dpp((int)(unsigned)(v & 0xffffffffLL), 0x128, 0xF, 0xF, true);  // row_ror:8
      const int hi2 = __builtin_amdgcn_mov_dpp((int)(v >> 32), 0x128, 0xF, 0xF, true);
      hh += __longlong_as_double((long long)(((unsigned long long)(unsigned)hi2 << 32) | (unsigned)lo2));
    }
    double hs[KK];   // (h h^T)[b][a], a = this lane's row (j; j & 1 when k = 2, two gene steps per pass); rotated
                     // (b = (j + r) & 3 at r) when KK = 4
#pragma unroll
    for (int b = 0; b < KK; ++b) hs[b] = __shfl(hh, 16 * (ROT ? ((j + b) & 3) : b) + (KK == 2 ? (j & 1) : j));
    // ---- F = A h^T (this lane's samples 4 cg + j in order, then the quad), E = W0 (h h^T), W rule; genes in
    // batches of SB steps (the H row block re-read from LDS per batch) to bound the live registers ----
    const double* const hrow = &sm.Hc[hb][j][0];   // H[a][4 cg + j] at hrow[16 cg + a]
    SOLO_STAMP(5);
#pragma unroll
    for (int s0 = 0; s0 < ((SKIP & 2) ? 0 : SOLO_S); s0 += SB) {
      double P[SB][KK];
      double h[KK], hn[KK];   // the next group's H loaded one step ahead
      asm volatile("" ::: "memory");   // re-read H per batch: holding all of it would spill A
#pragma unroll
      for (int a = 0; a < KK; ++a) h[a] = hrow[a];
#pragma unroll
      for (int cg = 0; cg < NCG; ++cg) {
        if (cg + 1 < NCG) {
#pragma unroll
          for (int a = 0; a < KK; ++a) hn[a] = hrow[16 * (cg + 1) + a];
        }
#pragma unroll
        for (int q = 0; q < SB; ++q)
#pragma unroll
          for (int a = 0; a < KK; ++a)   // the chain's first term is a product (fma onto +0 but for the zero's sign)
            P[q][a] = cg == 0 ? av(s0 + q, 0) * h[a] : fma(av(s0 + q, cg), h[a], P[q][a]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int a = 0; a < KK; ++a) h[a] = hn[a];
      }
      if constexpr (KK == 2) {
        // two gene steps per pass: lane j takes step s0 + q + (j >> 1), row a = j & 1 (lanes 2, 3 would idle)
#pragma unroll
        for (int q = 0; q < SB; q += 2) {
          const int s = s0 + q, t = s + 1;
          const bool hi = j >= 2;
          // F: reduce-scatter of (s, 0), (s, 1), (t, 0), (t, 1) over the quad; lane j ends with entry j
          // (every DPP read below runs with the whole quad active: no DPP under a lane-dependent branch)
          const double k0 = hi ? P[q + 1][0] : P[q][0], k1 = hi ? P[q + 1][1] : P[q][1];
          const double o0 = hi ? P[q][0] : P[q + 1][0], o1 = hi ? P[q][1] : P[q + 1][1];
          const double x0 = qdpp<0x4E>(o0), x1 = qdpp<0x4E>(o1);   // partner j ^ 2
          const double q0 = k0 + x0, q1 = k1 + x1;
          const double mine = (j & 1) ? q1 : q0, other = (j & 1) ? q0 : q1;
          const double y = qdpp<0xB1>(other);                       // partner j ^ 1
          const double f = mine + y;
          // this lane's W row: lanes 2, 3 take step t's values from lanes 0, 1
          const double wt = qdpp<0x44>(w_[t]);
          const double z = hi ? wt : w_[s];
          const double z0 = qdpp<0xA0>(z), z1 = qdpp<0xF5>(z);     // W0[g][0], W0[g][1]: lanes (j & 2), (j & 2) + 1
          const double e = fma(z1, hs[1], fma(z0, hs[0], 0.0));
          const double r = mu_rule_nb(z, f, e);
          const double rt = qdpp<0xEE>(r);                          // step t's result back to lanes 0, 1
          w_[s] = hi ? w_[s] : r;
          w_[t] = hi ? w_[t] : rt;
        }
      } else {
#pragma unroll
        for (int q = 0; q < SB; ++q) {
          const int s = s0 + q;
          double f = 0.0, e = 0.0;
          if constexpr (ROT) {
            // register r of lane j holds row (j + r) & 3: the quad sum of row j by three uniform rotations
            f = (P[q][0] + qdpp<0x4E>(P[q][2])) + (qdpp<0x39>(P[q][3]) + qdpp<0x93>(P[q][1]));
            e = fma(w_[s], hs[0], e);
            e = fma(qdpp<0x39>(w_[s]), hs[1], e);
            e = fma(qdpp<0x4E>(w_[s]), hs[2], e);
            e = fma(qdpp<0x93>(w_[s]), hs[3], e);
          } else {
#pragma unroll
            for (int a = 0; a < KK; ++a) {
              double v = P[q][a];
              v = v + qdpp<0xB1>(v);   // lanes j ^ 1
              v = v + qdpp<0x4E>(v);   // lanes j ^ 2
              f = (j == a) ? v : f;
            }
#pragma unroll
            for (int b = 0; b < KK; ++b) e = fma(qbcast(w_[s], b), hs[b], e);
          }
          if (j < KK) w_[s] = mu_rule_nb(w_[s], f, e);
        }
      }
    }
    SOLO_STAMP(6);
  }
  if ((SKIP & 64) && tid == 0 && prof)
    for (int i = 0; i < 8; ++i) prof[i] = pacc[i];
#undef SOLO_STAMP
  // ---- final factors and the stop state ----
#pragma unroll
  for (int s = 0; s < SOLO_S; ++s) {
    const int g = 128 * w + 16 * s + 4 * bq + K;
    if (g < m && j < kt) Wj[(long)j * lay.w_ld + g] = w_[s];
  }
  for (int x = tid; x < kt * n; x += 64 * SOLO_W) {
    const int c = x / kt, a = x - c * kt;
    Hj[(long)c * lay.h_sc + (long)a * lay.h_sa] = sm.Hc[hb][c][hp(c, a)];
  }
  if (tid == 0) {
    if constexpr (JOBS) {
      lay.stop_iter[rid] = sm.stop;
      lay.stop_reason[rid] = sm.reason;
    } else {
      state[0] = sm.stop;
      state[1] = sm.reason;
    }
  }
  }   // jobs
}

template <int NCG, int KK, int SKIP = 0, int SBO = 0, int SL = 0, bool JOBS = false>
__global__ __launch_bounds__(64 * SOLO_W) void k_solo_mu(const double* __restrict__ A, int m, int n,
                                                         double* __restrict__ W, double* __restrict__ H, int maxiter,
                                                         int stop_rule, int* __restrict__ state, int kt_arg,
                                                         long long* __restrict__ prof, SoloLayout lay) {
  __shared__ SoloSmem<NCG> sm;
  __shared__ SoloAl<NCG, SL> Al;
  solo_mu_body<NCG, KK, SKIP, SBO, SL, JOBS>(A, m, n, W, H, maxiter, stop_rule, state, kt_arg, prof, lay, sm, Al,
                                              (int)blockIdx.x, (int)gridDim.x);
}

// ---- ranks 5..8: the same one-workgroup design with the factor rows in two groups of four ----
// Lane layout as k_solo_mu; w_[s][h] = W[gene(s)][4 h + j] (zero past the restart's rank kt).  G = W^T A runs two
// 4x4x4 MFMA chains per (gene step, column group) -- rows 0..3 and 4..7 -- and W^T W three (rows 0-3 x 0-3,
// 0-3 x 4-7, 4-7 x 4-7; the fourth block is the transpose of the second, the same products in the same order).
// The register file cannot hold A beside these accumulators, so the last SL gene steps of A live in LDS, and each
// wave sums its four gene blocks b (lane bits 2..3, row rotations) before writing its partials: the LDS holds
// 16 doubles per (wave, chain) instead of 64.  F = A h^T and E = W0 (h h^T) run on 4x4x4 MFMAs too: the X operand
// is A's (W0's) block with the lane fields of gene and sample (factor) swapped -- a ds_bpermute for the steps in
// registers, a permuted LDS address for those in LDS -- and D lands in W's own layout, so the W rule is elementwise
// (a VALU form with quad reductions was 12 % slower: k-padding aside, its ~1 450 VALU instructions per lane per
// iteration cost more than the 4x4x4 MFMAs at ~25 cycles each).  Per iteration: MFMA chains -> block sums -> LDS |
// barrier | wave sums in order (one thread per entry) | barrier | H update | barrier | stop check (wave 0) + h h^T
// (three 4x4x4 chains over the 48 padded samples, every wave, into its own LDS copy), F / E / W rule by gene
// steps.  Every order is a function of (m, n, k) only.
constexpr int S8_CH = 3;   // W^T W chains

template <int NCG>
struct Solo8Smem {
  double Gp[SOLO_W][2 * NCG + S8_CH][16];   // block-summed partials, [chain][4 i + j] (i: row, j: column of the block)
  double Hc[2][SOLO_NCOLP][8];              // H by (sample, row), rows padded to 8: zero past k and n
  double Hh[SOLO_W][8][8];                  // h h^T, each wave's own copy
  double Gs[8][4 * NCG];                    // G = W^T A
  double WW[8][8];                          // W^T W
  int stop, reason;
};

// sum of the four gene blocks b (lane bits 2..3) by row rotations; lanes with b = 0 hold it
__device__ __forceinline__ double bsum4(double v) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)(u & 0xffffffffLL), 0x124, 0xF, 0xF, true);   // row_ror:4
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), 0x124, 0xF, 0xF, true);
  v += __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
  const long long t = __double_as_longlong(v);
  const int lo2 = __builtin_amdgcn_mov_dpp((int)(unsigned)(t & 0xffffffffLL), 0x128, 0xF, 0xF, true);  // row_ror:8
  const int hi2 = __builtin_amdgcn_mov_dpp((int)(t >> 32), 0x128, 0xF, 0xF, true);
  return v + __longlong_as_double((long long)(((unsigned long long)(unsigned)hi2 << 32) | (unsigned)lo2));
}

// SKIP != 0 only in tools/solobench.hip (phase costs): bit 0 no G / W^T W MFMAs, 1 no F / E / W rule, 2 no h h^T,
// 3 no stop check, 4 no wave sums, 5 no H update
template <int NCG, int SL, bool JOBS, int SKIP, int FMQ, bool ONE = false>
__device__ __forceinline__ void solo8_mu_body(const double* __restrict__ A, int m, int n, double* __restrict__ W,
                                              double* __restrict__ H, int maxiter, int stop_rule,
                                              int* __restrict__ state, int kt_arg, const SoloLayout& lay,
                                              Solo8Smem<NCG>& sm, SoloAl<NCG, SL>& Al, int jx0, int jstep) {
  constexpr int SR = SOLO_S - SL;       // gene steps of A in registers
  const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63, K = l >> 4,
            bq = (l >> 2) & 3, j = l & 3;
  double a_[SR > 0 ? SR : 1][NCG], w_[SOLO_S][2];
  auto av = [&](int s, int cg) -> double { return s < SR ? a_[s < SR ? s : 0][cg] : Al[s < SR ? 0 : s - SR][cg][tid]; };
#pragma unroll
  for (int s = 0; s < SOLO_S; ++s) {
    const int g = 128 * w + 16 * s + 4 * bq + K;
#pragma unroll
    for (int cg = 0; cg < NCG; ++cg) {
      const int c = 4 * cg + j;
      const double v = (g < m && c < n) ? A[(long)c * lay.a_ld + g] : 0.0;
      if (s < SR)
        a_[s < SR ? s : 0][cg] = v;
      else
        Al[s < SR ? 0 : s - SR][cg][tid] = v;
    }
  }
  const int njobs = JOBS ? lay.njobs : 1;
  for (int jx = JOBS ? jx0 : 0; jx < (ONE ? jx0 + 1 : njobs); jx += JOBS ? jstep : 1) {   // ONE: job jx0 only
  double* __restrict__ Wj = W;
  double* __restrict__ Hj = H;
  int kt = kt_arg, rid = -1;
  if constexpr (JOBS) {   // uniform job fields (scalar registers: the vector ones are A's)
    const nmfc::SoloJob jb = lay.jobs[__builtin_amdgcn_readfirstlane(jx)];
    const int col0 = __builtin_amdgcn_readfirstlane(jb.col0);
    Wj = W + (long)col0 * lay.w_ld;
    Hj = H + (long)col0 * lay.h_sa;
    kt = __builtin_amdgcn_readfirstlane(jb.k);
    rid = __builtin_amdgcn_readfirstlane(jb.rid);
  }
#pragma unroll
  for (int s = 0; s < SOLO_S; ++s) {
    const int g = 128 * w + 16 * s + 4 * bq + K;
#pragma unroll
    for (int h = 0; h < 2; ++h) w_[s][h] = (g < m && 4 * h + j < kt) ? Wj[(long)(4 * h + j) * lay.w_ld + g] : 0.0;
  }
  __syncthreads();   // the previous job's last reads of sm are done
  for (int x = tid; x < 2 * SOLO_NCOLP * 8; x += 64 * SOLO_W) (&sm.Hc[0][0][0])[x] = 0.0;
  if (tid == 0) {
    sm.stop = 0;
    sm.reason = 0;
  }
  __syncthreads();
  for (int x = tid; x < kt * n; x += 64 * SOLO_W) {
    const int c = x / kt, a = x - c * kt;
    sm.Hc[0][c][a] = Hj[(long)c * lay.h_sc + (long)a * lay.h_sa];
  }
  __syncthreads();
  int hb = 0;
  int cls = 0, unch = 0;   // wave 0: lane i's class, unchanged checks
  for (int iter = 1; maxiter >= 1 && iter <= maxiter + 1; ++iter) {
    // ---- this wave's partials of G = W^T A and W^T W (MFMA chains in gene order), gene blocks summed; the
    // column groups in two passes over the gene steps (half the accumulators live at a time) ----
    const int slot = 4 * K + j;   // D layout: lane 16 i + 4 b + j holds block b's [i][j]
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      constexpr int NH = (NCG + 1) / 2;
      const int cg0 = part * NH, cg1 = part ? NCG : NH;
      double acc[2][NH], ww[S8_CH];
#pragma unroll
      for (int c = 0; c < NH; ++c) acc[0][c] = acc[1][c] = 0.0;
#pragma unroll
      for (int c = 0; c < S8_CH; ++c) ww[c] = 0.0;
#pragma unroll
      for (int s = 0; s < ((SKIP & 1) ? 0 : SOLO_S); ++s) {
#pragma unroll
        for (int cg = cg0; cg < cg1; ++cg) {
          const double x = av(s, cg);
          acc[0][cg - cg0] = __builtin_amdgcn_mfma_f64_4x4x4f64(w_[s][0], x, acc[0][cg - cg0], 0, 0, 0);
          acc[1][cg - cg0] = __builtin_amdgcn_mfma_f64_4x4x4f64(w_[s][1], x, acc[1][cg - cg0], 0, 0, 0);
        }
        if (part == 0) {
          ww[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(w_[s][0], w_[s][0], ww[0], 0, 0, 0);
          ww[1] = __builtin_amdgcn_mfma_f64_4x4x4f64(w_[s][0], w_[s][1], ww[1], 0, 0, 0);
          ww[2] = __builtin_amdgcn_mfma_f64_4x4x4f64(w_[s][1], w_[s][1], ww[2], 0, 0, 0);
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int cg = cg0; cg < cg1; ++cg) {
          const double v = bsum4(acc[h][cg - cg0]);
          if (bq == 0) sm.Gp[w][h * NCG + cg][slot] = v;
        }
      if (part == 0) {
#pragma unroll
        for (int c = 0; c < S8_CH; ++c) {
          const double v = bsum4(ww[c]);
          if (bq == 0) sm.Gp[w][2 * NCG + c][slot] = v;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    if (sm.stop) break;   // decided at the previous iteration (its updates are done)
    // ---- sums over the waves in order: G (kt x n) and W^T W (kt x kt), one thread per entry ----
    // (tid through an empty asm: the index arithmetic of this phase, the H update and the stop check stays in
    // its phase instead of being hoisted out of the iteration loop into registers A needs)
    int tq = tid;
    asm volatile("" : "+v"(tq));
    for (int o = tq; !(SKIP & 16) && o < kt * n + kt * kt; o += 64 * SOLO_W) {
      int ch, idx, a, c;
      if (o < kt * n) {
        a = o / n;
        c = o - a * n;
        ch = (a >> 2) * NCG + (c >> 2);
        idx = 4 * (a & 3) + (c & 3);
      } else {
        a = (o - kt * n) / kt;
        c = (o - kt * n) - a * kt;
        const int ha = a >> 2, hc = c >> 2;
        ch = 2 * NCG + ha + hc;
        idx = ha > hc ? 4 * (c & 3) + (a & 3) : 4 * (a & 3) + (c & 3);   // rows 4-7 x 0-3: the transpose
      }
      double v = sm.Gp[0][ch][idx];
#pragma unroll
      for (int q = 1; q < SOLO_W; ++q) v += sm.Gp[q][ch][idx];
      if (o < kt * n)
        sm.Gs[a][c] = v;
      else
        sm.WW[a][c] = v;
    }
    __syncthreads();
    // ---- H update (nmf_mu.c:178-191): d = (W^T W) H summed over the rows in order ----
    const int nb = hb ^ 1;
    asm volatile("" : "+v"(tq));
    for (int x = tq; !(SKIP & 32) && x < kt * n; x += 64 * SOLO_W) {
      const int c = x / kt, a = x - c * kt;
      double d = 0.0;
      for (int b = 0; b < kt; ++b) d = fma(sm.WW[a][b], sm.Hc[hb][c][b], d);
      sm.Hc[nb][c][a] = mu_rule(sm.Hc[hb][c][a], sm.Gs[a][c], d);
    }
    __syncthreads();
    hb = nb;
    // ---- stop rule (nmf_mu.c:253-282), wave 0 ----
    if (w == 0) {
      const bool check = !(SKIP & 8) && stop_rule != nmfc::STOP_FIXED && iter > 1 && (iter % 2 == 0);
      int reason = 0;
      if (check) {
        bool ch = false;
        int lq = l;
        asm volatile("" : "+v"(lq));   // window addresses computed here, not held across the loop
        if (stop_rule == nmfc::STOP_REF_COMPAT) {
          if (lq < kt && lq < n) {   // window i reads the flat k x n column-major buffer at [i n, i n + k)
            int cl = 0;
            double prev = 0.0;
            for (int jj = 0; jj < kt; ++jj) {
              const int f = lq * n + jj, c = f / kt, a = f - c * kt;
              const double v = sm.Hc[hb][c][a];
              if (jj > 0 && v > prev) cl = jj;
              prev = v;
            }
            ch = cl != cls;
            cls = cl;
          }
        } else if (stop_rule == nmfc::STOP_ARGMAX_STABLE) {
          if (lq < n) {
            int best = 0;
            double bv = sm.Hc[hb][lq][0];
            for (int a = 1; a < kt; ++a) {
              const double v = sm.Hc[hb][lq][a];
              if (v > bv) {
                bv = v;
                best = a;
              }
            }
            ch = best != cls;
            cls = best;
          }
        }
        if (__ballot(ch) == 0) {
          if (++unch >= 200) reason = 1;   // nmf_mu.c:269-271
        } else {
          unch = 0;
        }
      }
      if (!reason && iter >= maxiter) reason = 2;
      if (reason && l == 0) {
        sm.stop = iter;
        sm.reason = reason;
      }
    }
    // ---- h h^T: three 4x4x4 chains over the padded samples (sample blocks b summed), into this wave's copy ----
    {
      int lq = l;
      asm volatile("" : "+v"(lq));
      const int hrow0 = 4 * ((lq >> 2) & 3) + (lq >> 4), hj = lq & 3;
      double hll = 0.0, hlh = 0.0, hhh = 0.0;
#pragma unroll
      for (int t = 0; t < ((SKIP & 4) ? 0 : SOLO_NCOLP / 16); ++t) {
        const double x0 = sm.Hc[hb][16 * t + hrow0][hj], x1 = sm.Hc[hb][16 * t + hrow0][4 + hj];
        hll = __builtin_amdgcn_mfma_f64_4x4x4f64(x0, x0, hll, 0, 0, 0);
        hlh = __builtin_amdgcn_mfma_f64_4x4x4f64(x0, x1, hlh, 0, 0, 0);
        hhh = __builtin_amdgcn_mfma_f64_4x4x4f64(x1, x1, hhh, 0, 0, 0);
      }
      hll = bsum4(hll);
      hlh = bsum4(hlh);
      hhh = bsum4(hhh);
      if (bq == 0) {   // lane 16 i + j: [i][j] of each block; rows 4-7 x 0-3 the transpose of rows 0-3 x 4-7
        sm.Hh[w][K][j] = hll;
        sm.Hh[w][K][4 + j] = hlh;
        sm.Hh[w][4 + j][K] = hlh;
        sm.Hh[w][4 + K][4 + j] = hhh;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    {
      // ---- F = A h^T and E = W0 (h h^T) on 4x4x4 MFMAs, W rule ----
      // X = A's (gene, sample) block with the two lane fields swapped (lane 16 kk + 4 b + i takes the value of lane
      // 16 i + 4 b + kk: ds_bpermute for the steps in registers, a permuted LDS address for those in LDS), Y = the
      // H^T block; D lands in W's own layout (lane 16 K + 4 b + j: gene 16 s + 4 b + K, row 4 h + j), so the rule
      // needs no reduction.  F chains over the column groups in order; E over the two row groups.
      const int tl = ((l & 3) << 4) | (l & 12) | (l >> 4);
      auto tperm = [&](double v) -> double {
        const long long u = __double_as_longlong(v);
        const int lo = __builtin_amdgcn_ds_bpermute(tl << 2, (int)(unsigned)(u & 0xffffffffLL));
        const int hi = __builtin_amdgcn_ds_bpermute(tl << 2, (int)(u >> 32));
        return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
      };
      double Y[NCG][2], Yh[2][2];   // H[4 h + j][4 t + K]; (h h^T)[4 g + K][4 h + j]
#pragma unroll
      for (int t = 0; t < NCG; ++t)
#pragma unroll
        for (int h = 0; h < 2; ++h) Y[t][h] = sm.Hc[hb][4 * t + K][4 * h + j];
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int h = 0; h < 2; ++h) Yh[g][h] = sm.Hh[w][4 * g + K][4 * h + j];
      constexpr int SQ = FMQ;   // gene steps whose chains run interleaved
#pragma unroll
      for (int s0 = 0; s0 < ((SKIP & 2) ? 0 : SOLO_S); s0 += SQ) {
        double f[SQ][2], e[SQ][2];
#pragma unroll
        for (int q = 0; q < SQ; ++q) {
          const double x0 = tperm(w_[s0 + q][0]), x1 = tperm(w_[s0 + q][1]);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            e[q][h] = __builtin_amdgcn_mfma_f64_4x4x4f64(x0, Yh[0][h], 0.0, 0, 0, 0);
            e[q][h] = __builtin_amdgcn_mfma_f64_4x4x4f64(x1, Yh[1][h], e[q][h], 0, 0, 0);
            f[q][h] = 0.0;
          }
        }
#pragma unroll
        for (int t = 0; t < NCG; ++t)
#pragma unroll
          for (int q = 0; q < SQ; ++q) {
            const int s = s0 + q;
            const double x = s < SR ? tperm(a_[s < SR ? s : 0][t]) : Al[s < SR ? 0 : s - SR][t][64 * w + tl];
#pragma unroll
            for (int h = 0; h < 2; ++h) f[q][h] = __builtin_amdgcn_mfma_f64_4x4x4f64(x, Y[t][h], f[q][h], 0, 0, 0);
          }
#pragma unroll
        for (int q = 0; q < SQ; ++q) {
          const int s = s0 + q;
          const double n0 = mu_rule_nb(w_[s][0], f[q][0], e[q][0]);
          w_[s][1] = mu_rule_nb(w_[s][1], f[q][1], e[q][1]);
          w_[s][0] = n0;
        }
      }
    }
  }
  // ---- final factors and the stop state ----
#pragma unroll
  for (int s = 0; s < SOLO_S; ++s) {
    const int g = 128 * w + 16 * s + 4 * bq + K;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (g < m && 4 * h + j < kt) Wj[(long)(4 * h + j) * lay.w_ld + g] = w_[s][h];
  }
  for (int x = tid; x < kt * n; x += 64 * SOLO_W) {
    const int c = x / kt, a = x - c * kt;
    Hj[(long)c * lay.h_sc + (long)a * lay.h_sa] = sm.Hc[hb][c][a];
  }
  if (tid == 0) {
    if constexpr (JOBS) {
      lay.stop_iter[rid] = sm.stop;
      lay.stop_reason[rid] = sm.reason;
    } else {
      state[0] = sm.stop;
      state[1] = sm.reason;
    }
  }
  }   // jobs
}

template <int NCG, int SL, bool JOBS, int SKIP = 0, int FMQ = JOBS ? 2 : 4>
__global__ __launch_bounds__(64 * SOLO_W) void k_solo8_mu(const double* __restrict__ A, int m, int n,
                                                          double* __restrict__ W, double* __restrict__ H, int maxiter,
                                                          int stop_rule, int* __restrict__ state, int kt_arg,
                                                          SoloLayout lay) {
  __shared__ Solo8Smem<NCG> sm;
  __shared__ SoloAl<NCG, SL> Al;
  solo8_mu_body<NCG, SL, JOBS, SKIP, FMQ>(A, m, n, W, H, maxiter, stop_rule, state, kt_arg, lay, sm, Al,
                                           (int)blockIdx.x, (int)gridDim.x);
}

// A batch's solo jobs of every kernel rank in ONE launch (the per-rank launches on streams of their own were
// serialised by the hardware queues they shared: C2's rank-2 launch started when the rank-4 one ended).  Each
// workgroup runs jobs jx = blockIdx.x, + gridDim.x, ...; per job the kernel rank picks the body, whose A, LDS and
// arithmetic are those of the per-rank kernel (the same bits as the drop-in's nmfc_mu_solo).  LDS: one buffer for
// the largest body.  A2..A8: the bodies' A steps in LDS at this NCG (0 where a rank does not occur).
template <int NCG>
constexpr int solo_sl(int kp) {   // A's gene steps in LDS by (column groups, kernel rank): dispatch()'s table
  return kp == 8 ? (NCG <= 4 ? 0 : NCG <= 6 ? 1 : NCG <= 8 ? 2 : 3) : kp == 4 ? (NCG <= 6 ? 0 : NCG <= 8 ? 1 : 2) : 0;
}
template <int NCG>
constexpr size_t solo_lds_bytes() {
  constexpr size_t a = sizeof(SoloSmem<NCG>), b = sizeof(Solo8Smem<NCG>);
  constexpr size_t s4 = ((a + 15) / 16) * 16 + sizeof(SoloAl<NCG, solo_sl<NCG>(4)>);
  constexpr size_t s8 = ((b + 15) / 16) * 16 + sizeof(SoloAl<NCG, solo_sl<NCG>(8)>);
  constexpr size_t s2 = ((a + 15) / 16) * 16 + sizeof(SoloAl<NCG, 0>);
  return s4 > s8 ? (s4 > s2 ? s4 : s2) : (s8 > s2 ? s8 : s2);
}
template <int NCG>
__global__ __launch_bounds__(64 * SOLO_W) void k_solo_batch(const double* __restrict__ A, int m, int n,
                                                            double* __restrict__ W, double* __restrict__ H,
                                                            int maxiter, int stop_rule, SoloLayout lay) {
  __shared__ double lds[solo_lds_bytes<NCG>() / sizeof(double)];
  auto run = [&](int jx) __attribute__((always_inline)) {
    const int k = __builtin_amdgcn_readfirstlane(lay.jobs[jx].k);
    const int kp = k >= 5 ? 8 : (k == 3 && NCG > 8) ? 4 : k;
    // (an empty asm with a memory clobber opens every arm: the bodies' identical A loads stay in their arms
    // instead of being hoisted above the branch, where all arms' A registers would be live at once)
    if (kp == 8) {
      asm volatile("" ::: "memory");
      auto& sm = *reinterpret_cast<Solo8Smem<NCG>*>(lds);
      auto& Al = *reinterpret_cast<SoloAl<NCG, solo_sl<NCG>(8)>*>(lds + (sizeof(Solo8Smem<NCG>) + 15) / 16 * 2);
      solo8_mu_body<NCG, solo_sl<NCG>(8), true, 0, 2, true>(A, m, n, W, H, maxiter, stop_rule, nullptr, 0, lay, sm, Al,
                                                              jx, 1);
    } else {
      auto& sm = *reinterpret_cast<SoloSmem<NCG>*>(lds);
      constexpr size_t off = (sizeof(SoloSmem<NCG>) + 15) / 16 * 2;
      if (kp == 4) {
        asm volatile("" ::: "memory");
        auto& Al = *reinterpret_cast<SoloAl<NCG, solo_sl<NCG>(4)>*>(lds + off);
        solo_mu_body<NCG, 4, 0, 0, solo_sl<NCG>(4), true, true>(A, m, n, W, H, maxiter, stop_rule, nullptr, 0, nullptr,
                                                                lay, sm, Al, jx, 1);
      } else if (kp == 3) {
        if constexpr (NCG <= 8) {
          asm volatile("" ::: "memory");
          auto& Al = *reinterpret_cast<SoloAl<NCG, 0>*>(lds + off);
          solo_mu_body<NCG, 3, 0, 0, 0, true, true>(A, m, n, W, H, maxiter, stop_rule, nullptr, 0, nullptr, lay, sm, Al,
                                                    jx, 1);
        }
      } else {
        asm volatile("" ::: "memory");
        auto& Al = *reinterpret_cast<SoloAl<NCG, 0>*>(lds + off);
        solo_mu_body<NCG, 2, 0, 0, 0, true, true>(A, m, n, W, H, maxiter, stop_rule, nullptr, 0, nullptr, lay, sm, Al,
                                                  jx, 1);
      }
    }
  };
  run((int)blockIdx.x);   // one job per workgroup: the grid is the job list
}

// one restart (nmfc_mu_solo), or one kernel rank's jobs of a batch on persistent workgroups (beside k_small_mu
// blocks): the per-rank kernels
template <int NCG, int SL>
hipError_t launch8(int grid, const double* A, int m, int n, double* W, double* H, int maxiter, int stop_rule, int* st,
                   int kt, const SoloLayout& lay, hipStream_t s) {
  if (lay.jobs)
    hipLaunchKernelGGL((k_solo8_mu<NCG, SL, true>), dim3(grid), dim3(64 * SOLO_W), 0, s, A, m, n, W, H, maxiter,
                       stop_rule, st, kt, lay);
  else
    hipLaunchKernelGGL((k_solo8_mu<NCG, SL, false>), dim3(grid), dim3(64 * SOLO_W), 0, s, A, m, n, W, H, maxiter,
                       stop_rule, st, kt, lay);
  return hipGetLastError();
}

template <int NCG, int KK, int SL = 0>
hipError_t launch(int grid, const double* A, int m, int n, double* W, double* H, int maxiter, int stop_rule, int* st,
                  int kt, const SoloLayout& lay, hipStream_t s) {
  if (lay.jobs)
    hipLaunchKernelGGL((k_solo_mu<NCG, KK, 0, 0, SL, true>), dim3(grid), dim3(64 * SOLO_W), 0, s, A, m, n, W, H, maxiter,
                       stop_rule, st, kt, nullptr, lay);
  else
    hipLaunchKernelGGL((k_solo_mu<NCG, KK, 0, 0, SL, false>), dim3(grid), dim3(64 * SOLO_W), 0, s, A, m, n, W, H,
                       maxiter, stop_rule, st, kt, nullptr, lay);
  return hipGetLastError();
}

// every kernel rank of a batch in one k_solo_batch launch, one workgroup per job
hipError_t dispatch_batch(const double* A, int m, int n, double* W, double* H, int maxiter, int stop_rule,
                          const SoloLayout& lay, hipStream_t s) {
  const int ncg = (n + 3) / 4;
  const dim3 grid(lay.njobs), block(64 * SOLO_W);
  if (ncg <= 4)
    hipLaunchKernelGGL((k_solo_batch<4>), grid, block, 0, s, A, m, n, W, H, maxiter, stop_rule, lay);
  else if (ncg <= 6)
    hipLaunchKernelGGL((k_solo_batch<6>), grid, block, 0, s, A, m, n, W, H, maxiter, stop_rule, lay);
  else if (ncg <= 8)
    hipLaunchKernelGGL((k_solo_batch<8>), grid, block, 0, s, A, m, n, W, H, maxiter, stop_rule, lay);
  else
    hipLaunchKernelGGL((k_solo_batch<10>), grid, block, 0, s, A, m, n, W, H, maxiter, stop_rule, lay);
  return hipGetLastError();
}

// the kernel rank for (n, k): k = 3 beyond n = 32 runs as k = 4 with a zero padding row; ranks 5..8 run on
// k_solo8_mu (the restart's own rank, zero rows past it)
int solo_rank(int n, int k) { return k >= 5 ? 8 : (k == 3 && (n + 3) / 4 > 8) ? 4 : k; }

// the (column groups, rank, A steps in LDS) instantiation for (n, kernel rank kp); grid workgroups
hipError_t dispatch(int grid, int kp, const double* A, int m, int n, double* W, double* H, int maxiter, int stop_rule,
                    int* st, int kt, const SoloLayout& lay, hipStream_t s) {
  // samples in column groups of 4: NCG = 4, 6, 8, 10 groups (n <= 16, 24, 32, 40)
  const int ncg = (n + 3) / 4;
  const int gi = ncg <= 4 ? 0 : ncg <= 6 ? 1 : ncg <= 8 ? 2 : 3;
  if (kp == 8) {   // ranks 5..8: A steps in LDS where the registers would not hold them beside the two row groups
    switch (gi) {
      case 0: return launch8<4, 0>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
      case 1: return launch8<6, 1>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
      case 2: return launch8<8, 2>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
      default: return launch8<10, 3>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
    }
  }
  switch (kp * 4 + gi) {
    case 8: return launch<4, 2>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
    case 9: return launch<6, 2>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
    case 10: return launch<8, 2>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
    case 11: return launch<10, 2>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
    case 12: return launch<4, 3>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
    case 13: return launch<6, 3>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
    case 14: return launch<8, 3>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
    case 16: return launch<4, 4>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
    case 17: return launch<6, 4>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
    case 18: return launch<8, 4, 1>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
    case 19: return launch<10, 4, 2>(grid, A, m, n, W, H, maxiter, stop_rule, st, kt, lay, s);
    default: return hipErrorInvalidValue;
  }
}

struct SoloCache {   // device copy of the last A (compared byte for byte), work buffer, pinned staging
  std::vector<double>* a = nullptr;   // no destructor: HIP may be torn down at exit
  int m = 0, n = 0;
  double* dA = nullptr;
  double* dwork = nullptr;   // [state (2 ints, 16 B) | W m x k | H k x n]
  double* pin = nullptr;     // pinned image of dwork
  size_t cap = 0;            // doubles in dwork / pin
  hipStream_t st = nullptr;
  int dev = -1;              // the HIP device every resource above lives on
};
std::mutex g_lock;
SoloCache g;

void cache_drop() {   // g_lock held: frees everything, so the next call starts from scratch
  if (g.st) (void)hipStreamSynchronize(g.st);
  if (g.dA) (void)hipFree(g.dA);
  if (g.dwork) (void)hipFree(g.dwork);
  if (g.pin) (void)hipHostFree(g.pin);
  if (g.st) (void)hipStreamDestroy(g.st);
  delete g.a;
  g.a = nullptr;
  g.dA = g.dwork = g.pin = nullptr;
  g.st = nullptr;
  g.cap = 0;
  g.m = g.n = 0;
  g.dev = -1;
}

int fail(const char* what, hipError_t e) {
  char buf[256];
  snprintf(buf, sizeof buf, "nmfc_mu_solo: %s: %s", what, hipGetErrorString(e));
  nmfc_set_error(buf);
  return -1;
}

}  // namespace

#define SCHECK(x)                                \
  do {                                           \
    hipError_t e_ = (x);                         \
    if (e_ != hipSuccess) return fail(#x, e_);   \
  } while (0)

// nmfc_nmf_mu_release (compat.hip): the device copy of A, the work buffer and the pinned staging
extern "C" void nmfc_solo_release() {
  std::lock_guard<std::mutex> lock(g_lock);
  cache_drop();
}

// every shape with 2 <= k <= 8, k <= m <= 1024, k <= n <= 40 (ranks 5..8 on k_solo8_mu, A's last one to three
// gene steps in LDS by n).  Ranks 2..4 by (k, column groups of 4 samples):
// A fully in registers where that does not spill (k = 2; k = 3 to n = 32; k = 4 to n = 24); else the last
// steps of A in LDS (k = 4: one step to n = 32, two to n = 40) and k = 3 beyond n = 32 as k = 4 with a zero
// padding row (the rows of a restart never mix, so its bits are those of the unpadded arithmetic)
extern "C" int nmfc_mu_solo_fits(int m, int n, int k) {
  return m >= k && n >= k && k >= 2 && k <= 8 && m <= SOLO_MMAX && n <= SOLO_NMAX;
}

namespace {
int mu_solo_call(const double* A, int m, int n, int k, int maxiter, int stop_rule, const double* W0, const double* H0,
                 double* W, double* H, int* iters, int* early);
}

// The device copy of A, the work buffer, the pinned staging and the stream are kept across calls (nmf.r calls
// nmf_mu once per restart on one matrix) on the device of the call that made them: a call on another device, a
// failed call (nothing cached may hold a half-done upload) and NMFC_NMF_MU_CACHE=0 (after the call) free them.
extern "C" int nmfc_mu_solo(const double* A, int m, int n, int k, int maxiter, int stop_rule, const double* W0,
                            const double* H0, double* W, double* H, int* iters, int* early) {
  if (!A || !W0 || !H0 || !W || !H || !nmfc_mu_solo_fits(m, n, k) || maxiter < 0 ||
      (stop_rule != NMFC_STOP_FIXED && stop_rule != NMFC_STOP_REF_COMPAT && stop_rule != NMFC_STOP_ARGMAX_STABLE)) {
    nmfc_set_error("nmfc_mu_solo: bad arguments (needs 2 <= k <= 8, k <= m <= 1024, k <= n <= 40)");
    return -1;
  }
  std::lock_guard<std::mutex> lock(g_lock);
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return fail("hipGetDevice", hipErrorInvalidDevice);
  if (g.dev >= 0 && g.dev != dev) cache_drop();
  const int rc = mu_solo_call(A, m, n, k, maxiter, stop_rule, W0, H0, W, H, iters, early);
  const char* env = getenv("NMFC_NMF_MU_CACHE");
  if (rc != 0 || (env && atoi(env) == 0))
    cache_drop();
  else
    g.dev = dev;
  return rc;
}

namespace {
int mu_solo_call(const double* A, int m, int n, int k, int maxiter, int stop_rule, const double* W0, const double* H0,
                 double* W, double* H, int* iters, int* early) {
  const int kp = solo_rank(n, k);   // the kernel's rank (k = 3 padded to 4 at n > 32)
  const size_t la = (size_t)m * n, lw = (size_t)m * kp, lh = (size_t)kp * n;
  if (!g.st) SCHECK(hipStreamCreateWithFlags(&g.st, hipStreamNonBlocking));
  if (!(g.dA && g.m == m && g.n == n && memcmp(g.a->data(), A, la * sizeof(double)) == 0)) {
    if (g.dA) (void)hipFree(g.dA);
    g.dA = nullptr;
    delete g.a;
    g.a = new std::vector<double>(A, A + la);
    g.m = m;
    g.n = n;
    SCHECK(hipMalloc(&g.dA, la * sizeof(double)));
    SCHECK(hipMemcpyAsync(g.dA, A, la * sizeof(double), hipMemcpyHostToDevice, g.st));
  }
  const size_t need = 2 + lw + lh;
  if (g.cap < need) {
    if (g.dwork) (void)hipFree(g.dwork);
    if (g.pin) (void)hipHostFree(g.pin);
    g.dwork = g.pin = nullptr;
    g.cap = 0;
    SCHECK(hipMalloc(&g.dwork, need * sizeof(double)));
    SCHECK(hipHostMalloc(&g.pin, need * sizeof(double), hipHostMallocDefault));
    g.cap = need;
  }
  if (kp == k) {
    memcpy(g.pin + 2, W0, lw * sizeof(double));
    memcpy(g.pin + 2 + lw, H0, lh * sizeof(double));
  } else {   // W0 m x k -> m x kp with zero columns, H0 k x n -> kp x n with zero rows
    memcpy(g.pin + 2, W0, (size_t)m * k * sizeof(double));
    memset(g.pin + 2 + (size_t)m * k, 0, (size_t)m * (kp - k) * sizeof(double));
    for (int c = 0; c < n; ++c)
      for (int a = 0; a < kp; ++a) g.pin[2 + lw + (size_t)c * kp + a] = a < k ? H0[(size_t)c * k + a] : 0.0;
  }
  SCHECK(hipMemcpyAsync(g.dwork + 2, g.pin + 2, (lw + lh) * sizeof(double), hipMemcpyHostToDevice, g.st));
  int* dstate = reinterpret_cast<int*>(g.dwork);
  double* dW = g.dwork + 2;
  double* dH = dW + lw;
  const SoloLayout lay{m, m, kp, 1, nullptr, nullptr, nullptr, 1};
  SCHECK(dispatch(1, kp, g.dA, m, n, dW, dH, maxiter, stop_rule, dstate, k, lay, g.st));
  SCHECK(hipMemcpyAsync(g.pin, g.dwork, need * sizeof(double), hipMemcpyDeviceToHost, g.st));
  SCHECK(hipStreamSynchronize(g.st));
  int hstate[2];
  memcpy(hstate, g.pin, sizeof hstate);
  memcpy(W, g.pin + 2, (size_t)m * k * sizeof(double));   // the first k columns of the m x kp W
  if (kp == k) {
    memcpy(H, g.pin + 2 + lw, lh * sizeof(double));
  } else {
    for (int c = 0; c < n; ++c)
      for (int a = 0; a < k; ++a) H[(size_t)c * k + a] = g.pin[2 + lw + (size_t)c * kp + a];
  }
  if (iters) *iters = maxiter == 0 ? 0 : hstate[0];
  if (early) *early = hstate[1] == 1;
  return 0;
}
}  // namespace

// Batched form (nmfc_engine_run, small shapes), reading the engine's column-major Acm and the stacked W/H at each
// job's col0, stop state into stop_iter / stop_reason[rid]:
//   kp == 0: the solo jobs of every kernel rank (solo_rank(n, k)) in ONE k_solo_batch launch, one workgroup per
//            job in list order (the engine lists the costliest ranks first) -- the batch has the GPU to itself;
//   kp > 0:  the jobs of kernel rank kp on min(njobs, max_wgs) persistent workgroups running their jobs one after
//            another (beside k_small_mu blocks, which must not wait for CUs behind solo workgroups).
// Returns 0 or -1 (nmfc_last_error).
__attribute__((visibility("hidden"))) int nmfc_solo_batch_rank(int n, int k) { return solo_rank(n, k); }

__attribute__((visibility("hidden"))) int nmfc_solo_batch_launch(const double* Acm, long a_ld, int m, int n, double* W,
                                                                 long w_ld, double* H, long h_ld,
                                                                 const nmfc::SoloJob* djobs, int njobs, int kp,
                                                                 int maxiter, int stop_rule, int* stop_iter,
                                                                 int* stop_reason, int max_wgs, hipStream_t st) {
  if (njobs <= 0) return 0;
  if (!nmfc_mu_solo_fits(m, n, 2) || kp < 0 || kp == 1 || (kp > 4 && kp != 8)) {
    nmfc_set_error("nmfc_solo_batch_launch: shape outside the solo kernel's range");
    return -1;
  }
  const SoloLayout lay{a_ld, w_ld, 1, h_ld, djobs, stop_iter, stop_reason, njobs};
  if (kp == 0) {
    SCHECK(dispatch_batch(Acm, m, n, W, H, maxiter, stop_rule, lay, st));
  } else {
    const int grid = std::max(1, std::min(njobs, max_wgs > 0 ? max_wgs : njobs));
    SCHECK(dispatch(grid, kp, Acm, m, n, W, H, maxiter, stop_rule, nullptr, kp, lay, st));
  }
  return 0;
}
